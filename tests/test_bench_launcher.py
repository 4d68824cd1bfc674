"""bench.py's --gpus N launcher (CPU): the parent starts N rank processes with
torchrun's environment, rank 0's single JSON line is the output, a failing rank
ends the job with its status; the CPU-baseline thread count follows the
process's CPU share."""
import json
import os
import subprocess
import sys
import textwrap

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rank_envs_are_torchrun_like():
    envs = bench.rank_envs(4, 29555, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
               and e["PATH"] == "/bin" for e in envs)


def _run_spawn(tmp_path, body, n):
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(body))
    drv = (f"import sys; sys.path.insert(0, {REPO!r}); import bench; "
           f"sys.exit(bench.spawn_ranks({n}, ['--gpus', '{n}'], script={str(script)!r}))")
    env = dict(os.environ, HONK_BENCH_ONE_GPU="1")
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-c", drv], env=env, capture_output=True, text=True, timeout=120)


def test_spawn_two_ranks_one_json_line(tmp_path):
    body = """
        import json, os, sys
        import torch.distributed as dist
        dist.init_process_group("gloo")
        r, w = dist.get_rank(), dist.get_world_size()
        assert int(os.environ["LOCAL_RANK"]) == r
        sys.path.insert(0, os.environ.get("REPO_ROOT", "."))
        import torch
        t = torch.tensor([float(r + 1)])
        dist.all_reduce(t)
        print(f"rank {r} progress", file=sys.stderr)
        if r == 0:
            print(json.dumps({"n_gpus": w, "sum": float(t.item()), "argv": sys.argv[1:]}))
        dist.barrier()
        dist.destroy_process_group()
    """
    p = _run_spawn(tmp_path, body, 2)
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["sum"] == 3.0 and d["argv"] == ["--gpus", "2"]


def test_spawn_failing_rank_ends_job(tmp_path):
    body = """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)   # would wait for rank 1 forever in a real collective
    """
    p = _run_spawn(tmp_path, body, 2)
    assert p.returncode == 3


def test_cpu_share_bounded():
    n = bench.cpu_share()
    assert 1 <= n <= (os.cpu_count() or 1)
    old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        assert bench.cpu_share() == 1
    finally:
        if old is None:
            del os.environ["OMP_NUM_THREADS"]
        else:
            os.environ["OMP_NUM_THREADS"] = old


def test_train_flops_res26_narrow():
    from honk_amd import model as hm
    cfg = dict(hm.find_config("res26-narrow"))
    # 157.33 MFLOP forward, training ~3x forward - conv0 dgrad ~ 471 MFLOP
    assert abs(bench.train_flops_per_clip(cfg) / 1e6 - 471) < 2


def _fake_topology(root, gfx_versions):
    for i, v in enumerate(gfx_versions):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if v else 16}\nsimd_count {1024 if v else 0}\n"
                                      f"gfx_target_version {v}\n")


def test_count_gpus_sysfs(tmp_path):
    _fake_topology(tmp_path, [0, 90500, 90500, 90500])
    assert bench.count_gpus_sysfs(str(tmp_path), env={}) == 3
    assert bench.count_gpus_sysfs(str(tmp_path), env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.count_gpus_sysfs(str(tmp_path), env={"ROCR_VISIBLE_DEVICES": "2"}) == 1
    assert bench.count_gpus_sysfs(str(tmp_path / "missing"), env={}) is None


def test_spawn_parent_never_initialises_hip(tmp_path):
    """The --gpus N parent counts GPUs from sysfs only: with every torch.cuda entry
    that could reach the HIP runtime (amdsmi path included) made to fail, the parent
    still launches the ranks and torch.cuda stays uninitialised in it; too few GPUs
    in the topology end the job with status 2 before any rank starts."""
    topo = tmp_path / "topo"
    _fake_topology(topo, [0, 90500, 90500])
    script = tmp_path / "rank.py"
    script.write_text("import os, sys\nprint('{\"rank\": %s}' % os.environ['RANK'])\n")
    drv = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        import torch
        def _boom(*a, **k):
            raise AssertionError("HIP touched by the launcher")
        torch.cuda.device_count = _boom
        torch.cuda.is_available = _boom
        torch.cuda._lazy_init = _boom
        torch._C._cuda_getDeviceCount = _boom
        import bench
        rc = bench.spawn_ranks(int(sys.argv[1]), ['--gpus', sys.argv[1]], script={str(script)!r})
        assert not torch.cuda.is_initialized()
        sys.exit(rc)
    """)
    env = dict(os.environ, HONK_KFD_TOPOLOGY=str(topo))
    for k in ("HONK_BENCH_ONE_GPU", "WORLD_SIZE", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
              "CUDA_VISIBLE_DEVICES"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-c", drv, "2"], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip() == '{"rank": 0}'
    p = subprocess.run([sys.executable, "-c", drv, "3"], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, p.stderr
    assert "only 2 visible GPU(s)" in p.stderr


def test_modes_summary_keeps_every_number():
    """The bench line ends with a compact per-mode summary."""
    import bench
    res = {"dtype": "f16x2", "value": 3.0e5, "roofline": {"frac": 0.45},
           "bf16x3_mode": {"dtype": "bf16x3", "value": 1.9e5, "roofline": {"frac": 0.44}},
           "f32_mode": {"dtype": "f32", "value": 5.7e4, "roofline": {"frac": 0.7}},
           "c2_cnn_trad_pool2": {"f32_mode": {"value": 5.8e5, "dtype": "f32", "roofline": {"frac": 0.71}},
                                 "bf16x3_mode": {"value": 1.6e6, "dtype": "bf16x3", "roofline": {"frac": 0.4}}},
           "c3_res8_bf16": {"value": 7e6, "dtype": "bf16", "roofline": {"frac": 0.28}},
           "c5_res26_narrow_train": {"value": 1.26e5, "dtype": "f32", "roofline": {"frac": 0.38}},
           "cpu_baseline": {"value": 97.3, "cores": 16}}
    m = bench.modes_summary(res, "res15")
    assert m["res15_f16x2 (headline)"] == {"value": 3.0e5, "dtype": "f16x2", "frac": 0.45}
    assert set(m) == {"res15_f16x2 (headline)", "res15_bf16x3", "res15_f32", "c2_cnn-trad-pool2_f32",
                      "c2_cnn-trad-pool2_bf16x3", "c3_res8_bf16", "c5_res26_narrow_train", "cpu_baseline"}
    assert bench._plan_str(["block16p_kernel"] * 6 + ["block16l_kernel"]) == "block16p_kernel x6 + block16l_kernel x1"

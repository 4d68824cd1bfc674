"""Experiment builds for C3 (res8 bf16): patches to copies of csrc, full res.hip compile.
    python exp/c3_exp.py build VARIANT ...   -> exp/_c3/<variant>/libhonk_hip.so
    python exp/c3_exp.py time VARIANT ...    (GPU box: rocprofv3 kernel stats, res8 bf16 131072 clips)
Ablation variants compute wrong results (timing only); every access stays in bounds."""
import csv
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exp", "_c3")
VARIANTS = {
    "base": [],
    "norelu": [("res.hip", "        for (int r = 0; r < 4; ++r) pacc[n][r] += relu_keepnan(acc[r]);",
                "        for (int r = 0; r < 4; ++r) pacc[n][r] += acc[r];")],
    "nostage": [("res.hip", "      for (int u = 0; u < 4; ++u) put(r, c + u, v[u]);", "      for (int u = 0; u < 1; ++u) (void)v;")],
    "nozero": [("res.hip", "    for (int i = threadIdx.x; i < n16; i += 256) ((u32x4*)c0lds)[i] = u32x4{0u, 0u, 0u, 0u};", "    (void)n16;")],
    "c0noread": [("res.hip", "      for (int j = 0; j < 8; ++j) bv[j] = *(const unsigned short*)(la[j] + moff);",
                  "      for (int j = 0; j < 8; ++j) bv[j] = (unsigned short)(size_t)(la[j] + moff);")],
    "c0nomfma": [("res.hip", """        const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[n]),
                                                                  __builtin_bit_cast(bf16x8, b),
                                                                  f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);""",
                  """        const f32x4 acc = __builtin_bit_cast(f32x4, wa[n] ^ b);""")],
    "c0nostore": [("res.hip", "    if (q0 >= npo) continue;\n    char* op = oc + (size_t)q0 * CB;",
                   "    if (q0 >= npo || clip >= 0) { for (int n = 0; n < NT; ++n) asm volatile(\"\" :: \"v\"(pacc[n])); continue; }\n    char* op = oc + (size_t)q0 * CB;")],
    "pairw": [],
    "c0lb8": [("res.hip", "__global__ __launch_bounds__(256) void conv0m_kernel(", "__global__ __launch_bounds__(256, 8) void conv0m_kernel(")],
    "c0lb7": [("res.hip", "__global__ __launch_bounds__(256) void conv0m_kernel(", "__global__ __launch_bounds__(256, 7) void conv0m_kernel(")],
    "net": [],
    "net15": [("CFLAGS", "-DHONK_NET_ABL=15", "")],
    "net7": [("CFLAGS", "-DHONK_NET_ABL=7", "")],
    "pairB": [("res.hip", "(FM == 1 || (L.W >= 32 && L.L >= 3 &&", "(FM == 1 || (L.W >= 8 && L.L >= 3 &&")],
    "pairT": [("res_bf16p.inc", "  constexpr bool TBL = FM == 2;", "  constexpr bool TBL = FM == 2 || (FM == 0 && NS == 1);"),
              ("res_bf16p.inc", "  constexpr int PD = (FM == 2 && KSA % 7 == 0) ? 6 : G::PD;",
               "  constexpr int PD = ((FM == 2 || (FM == 0 && NS == 1)) && KSA % 7 == 0) ? 6 : G::PD;"),
              ("res_bf16p.inc", "  return FM == 2 ? g16p_zb_tbl()", "  return FM != 1 ? g16p_zb_tbl()"),
              ("res.hip", "(FM == 1 || (L.W >= 32 && L.L >= 3 &&", "(FM == 1 || (L.W >= 8 && L.L >= 3 &&")],
    "nodpp": [("res_bf16r.inc", "          for (int k = 0; k < 4; ++k) c[k] = sum16_dpp(csum[n][k]);",
               "          for (int k = 0; k < 4; ++k) c[k] = csum[n][k];")],
}


def build(name):
    d = os.path.join(OUT, name)
    src = os.path.join(d, "src")
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    shutil.copytree(os.path.join(ROOT, "honk_amd", "csrc"), os.path.join(src, "honk_amd", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(src, "include"))
    csrc = os.path.join(src, "honk_amd", "csrc")
    cflags = []
    for fn, a, b in VARIANTS[name]:
        if fn == "CFLAGS":
            cflags.append(a)
            continue
        f = os.path.join(csrc, fn)
        s = open(f).read()
        assert a in s, (name, fn, a[:80])
        open(f, "w").write(s.replace(a, b))
    obj = os.path.join(d, "res.o")
    cc = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-function",
          "-I", os.path.join(src, "include")]
    subprocess.run(cc + cflags + ["-c", os.path.join(csrc, "res.hip"), "-o", obj], check=True)
    bd = os.path.join(ROOT, "honk_amd", "_build")
    others = [os.path.join(bd, x + ".o") for x in ("runtime", "cnn", "train", "mfcc", "head", "augment")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(d, "libhonk_hip.so"), obj] + others, check=True)
    shutil.rmtree(src)
    os.remove(obj)
    return name


RUN = os.path.join(ROOT, "exp", "c3_prof.py")


ENV = {"pairw": {"HONK_RES_KERNEL": "w"}, "net": {"HONK_RES_KERNEL": "n"}, "net15": {"HONK_RES_KERNEL": "n"},
       "net7": {"HONK_RES_KERNEL": "n"}}


def time_variants(names):
    for name in names:
        od = os.path.join(ROOT, "gpurun_out", "c3", name)
        os.makedirs(od, exist_ok=True)
        env = dict(os.environ, HONK_LIB=os.path.join(OUT, name if name not in ("pairw", "net") else "base", "libhonk_hip.so"),
                   **ENV.get(name, {}))
        r = subprocess.run(["timeout", "-k", "10", "120", "rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv",
                            "-d", od, "-o", "run", "--", sys.executable, RUN], env=env, capture_output=True, text=True)
        if r.returncode != 0:
            print(name, "FAILED", r.returncode, r.stderr[-1500:], flush=True)
            sys.exit(r.returncode)
        f = glob.glob(os.path.join(od, "**", "*kernel_stats.csv"), recursive=True)[0]
        row = []
        for rec in csv.DictReader(open(f)):
            if "honk" in rec["Name"]:
                nm = rec["Name"].replace("void honk::res::", "").split("(")[0]
                row.append(f"{nm} {float(rec['AverageNs']) / 1e3:.1f}")
        print(f"{name:10s} " + " | ".join(row[:5]), flush=True)


if __name__ == "__main__":
    cmd, names = sys.argv[1], sys.argv[2:] or list(VARIANTS)
    if cmd == "build":
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(min(len(names), 5)) as ex:
            for n in ex.map(build, names):
                print("built", n, flush=True)
    else:
        time_variants(names)

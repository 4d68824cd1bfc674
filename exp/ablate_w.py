"""Timing-only ablation builds of the weight-stationary res kernel (res_bf16w.inc):
patched copies of the sources -> exp/_abl/<variant>/libhonk_hip.so (load with
HONK_LIB=...).  Variants give WRONG results by construction; never shipped."""
import os, shutil, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exp", "_abl")
NEVER = "a.TH == 12345"  # a runtime-false condition the compiler cannot fold

PATCHES = {
    "base": [],
    "nodma": [("__builtin_amdgcn_raw_ptr_buffer_load_lds(rs,", f"if ({NEVER}) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs,")],
    "nostore": [("__builtin_amdgcn_raw_buffer_store_b128(u32x4{lo[0], lo[1], hi[0], hi[1]}, out_p,",
                 f"if ({NEVER}) __builtin_amdgcn_raw_buffer_store_b128(u32x4{{lo[0], lo[1], hi[0], hi[1]}}, out_p,"),
                ("__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h[pt][NT - 1]), out_p,",
                 f"if ({NEVER}) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h[pt][NT - 1]), out_p,")],
    "nores": [("      if constexpr (RES && S == KR) res_loads(rr, po);", f"      if constexpr (RES && S == KR) if ({NEVER}) res_loads(rr, po);")],
    "noepi": [("        if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S) epi_step(ec);",
               f"        if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S) if ({NEVER}) epi_step(ec);"),
              ("      if constexpr (RES && S == KR) res_loads(rr, po);", f"      if constexpr (RES && S == KR) if ({NEVER}) res_loads(rr, po);")],
}
PATCHES["mfma"] = PATCHES["nodma"] + PATCHES["noepi"]

def build(name):
    d = os.path.join(OUT, name)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(os.path.join(d, "honk_amd"))
    shutil.copytree(os.path.join(ROOT, "honk_amd", "csrc"), os.path.join(d, "honk_amd", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
    f = os.path.join(d, "honk_amd", "csrc", "res_bf16w.inc")
    s = open(f).read()
    for a, b in PATCHES[name]:
        assert a in s, (name, a)
        s = s.replace(a, b)
    open(f, "w").write(s)
    obj = os.path.join(d, "res.o")
    cc = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(d, "include")]
    subprocess.run(cc + ["-c", os.path.join(d, "honk_amd", "csrc", "res.hip"), "-o", obj], check=True)
    bd = os.path.join(ROOT, "honk_amd", "_build")
    others = [os.path.join(bd, x) for x in ("runtime.o", "cnn.o", "train.o", "mfcc.o")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(d, "libhonk_hip.so"), obj] + others, check=True)
    shutil.rmtree(os.path.join(d, "honk_amd")); shutil.rmtree(os.path.join(d, "include")); os.remove(obj)
    return name

if __name__ == "__main__":
    from concurrent.futures import ThreadPoolExecutor
    names = sys.argv[1:] or list(PATCHES)
    with ThreadPoolExecutor(4) as ex:
        for n in ex.map(build, names):
            print("built", n, flush=True)

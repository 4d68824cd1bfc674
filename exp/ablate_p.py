"""Timing-only ablation builds of the fused pair kernel (res_bf16p.inc): patched
copies of the sources -> exp/_abl/p_<variant>/libhonk_hip.so (load with
HONK_LIB=...).  Variants give WRONG results by construction; never shipped."""
import os, shutil, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exp", "_abl")
NEVER = "a.H == 12345"  # a runtime-false condition the compiler cannot fold

EPI = ("        if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S) epi_step(rolec, ec);",
       f"        if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S) if ({NEVER}) epi_step(rolec, ec);")
RES = ("      if constexpr (ISB && S == 0) res_loads(cur.pix);", f"      if constexpr (ISB && S == 0) if ({NEVER}) res_loads(cur.pix);")
DMA = ("        dma(widx ? roff[rb] : roff[ra],", f"        if ({NEVER}) dma(widx ? roff[rb] : roff[ra],")
BAR = ("      __builtin_amdgcn_s_barrier();\n      // the first m-tile", "      if (" + NEVER + ") __builtin_amdgcn_s_barrier();\n      // the first m-tile")
GEO = [("      if constexpr (S == KW) walk_adv(wk);", "      if constexpr (S == KW) if (" + NEVER + ") walk_adv(wk);"),
       ("      if constexpr (S == KG) nxt = geo(wk);", "      if constexpr (S == KG) nxt = cur;")]
BCAST = [("    return base + (int)(e & 0x7fu);\n  };", "    return zoff + (base & 0) + (int)(e & 0x7fu);\n  };")]
PATCHES = {
    "base": [],
    "nobar": [BAR],
    "nodma": [DMA],
    "noepi": [EPI, RES],
    "nogeo": GEO,
    "mfma": [DMA, EPI, RES, BAR],
    "bcast": BCAST,
    "nosb": [("      __builtin_amdgcn_sched_barrier(0);\n      const u32x4 (&ac)[SP]", "      const u32x4 (&ac)[SP]")],
    "aonly": [("        if (it == 0) run_mtile(rolec,", "        if (ISB && a.H != 12345) { for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f}; } else if (it == 0) run_mtile(rolec,"),
              ("        else run_mtile(rolec, std::integral_constant<bool, false>{}", "        else if (!(ISB && a.H != 12345)) run_mtile(rolec, std::integral_constant<bool, false>{}")],
    "bonly": [("        if (it == 0) run_mtile(rolec,", "        if (!ISB && a.H != 12345) { for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f}; } else if (it == 0) run_mtile(rolec,"),
              ("        else run_mtile(rolec, std::integral_constant<bool, false>{}", "        else if (!(!ISB && a.H != 12345)) run_mtile(rolec, std::integral_constant<bool, false>{}")],
}

def build(name):
    d = os.path.join(OUT, "p_" + name)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(os.path.join(d, "honk_amd"))
    shutil.copytree(os.path.join(ROOT, "honk_amd", "csrc"), os.path.join(d, "honk_amd", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
    f = os.path.join(d, "honk_amd", "csrc", "res_bf16p.inc")
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

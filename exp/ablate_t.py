"""Timing-only ablation builds of the MFMA training conv (train.hip conv3x3m_kernel):
patched copies -> exp/_abl/t_<variant>/libhonk_hip.so.  WRONG results by construction."""
import os, shutil, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exp", "_abl")
NEVER = "a.H == 12345"
PATCHES = {
    "nostage": [("      xl[c * PS + rc] = (h >= 0", f"      if ({NEVER}) xl[c * PS + rc] = (h >= 0")],
    "nostore": [("            if (o < C) yb[(size_t)o * a.H * a.W + pix] = acc[n][i];",
                 f"            if (o < C && {NEVER}) yb[(size_t)o * a.H * a.W + pix] = acc[n][i];")],
}
PATCHES["mfma"] = PATCHES["nostage"] + PATCHES["nostore"]

def build(name):
    d = os.path.join(OUT, "t_" + name)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(os.path.join(d, "honk_amd"))
    shutil.copytree(os.path.join(ROOT, "honk_amd", "csrc"), os.path.join(d, "honk_amd", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
    f = os.path.join(d, "honk_amd", "csrc", "train.hip")
    s = open(f).read()
    for a, b in PATCHES[name]:
        assert a in s, (name, a)
        s = s.replace(a, b)
    open(f, "w").write(s)
    obj = os.path.join(d, "train.o")
    cc = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(d, "include")]
    subprocess.run(cc + ["-c", f, "-o", obj], check=True)
    bd = os.path.join(ROOT, "honk_amd", "_build")
    others = [os.path.join(bd, x) for x in ("runtime.o", "cnn.o", "res.o", "mfcc.o")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(d, "libhonk_hip.so"), obj] + others, check=True)
    shutil.rmtree(os.path.join(d, "honk_amd")); shutil.rmtree(os.path.join(d, "include")); os.remove(obj)
    return name

if __name__ == "__main__":
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(3) as ex:
        for n in ex.map(build, sys.argv[1:] or list(PATCHES)):
            print("built", n, flush=True)

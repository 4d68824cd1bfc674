"""Experiment builds of the f16x2 res15 pair kernel (block16p_kernel<3, 1, 4, 4, 1, 2>).

    python exp/pair_exp.py build VARIANT ...     -> exp/_pair/<variant>/libhonk_hip.so
    python exp/pair_exp.py time VARIANT ...      (GPU box: rocprofv3 kernel stats per variant)

A variant = patches to a copy of csrc/res_bf16p.inc (and res.hip), compiled with every
kernel instantiation the f16x2 res15 forward does not launch cut out of the copy's
res.hip (the "reduce" patches: ~5x faster to compile).  Ablation variants compute WRONG
results by construction (timing only, never shipped); every memory access stays in
bounds (skipped work, frozen geometry), so they are as safe to run as the product.
"""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "exp", "_pair")
NEVER = "a.H == 12345"  # runtime-false: the compiler keeps the code shape around it

REDUCE = [
    ("""  HONK_W(1, 0) HONK_W(2, 0) HONK_W(3, 0)
  HONK_W(1, 1) HONK_W(2, 1) HONK_W(3, 1)
  HONK_W(1, 2) HONK_W(2, 2) HONK_W(3, 2)""", "  HONK_W(3, 2)"),
    ("""  if (SP == 1) {
    if (p.NT == 1 && p.MT == g16r_mt(1, 1)) return launch_block16r<1, g16r_mt(1, 1), 1>(a, st);
    if (p.NT == 2 && p.MT == g16r_mt(2, 1)) return launch_block16r<2, g16r_mt(2, 1), 1>(a, st);
    if (p.NT == 3 && p.MT == g16r_mt(3, 1)) return launch_block16r<3, g16r_mt(3, 1), 1>(a, st);
  } else {
    if (p.NT == 1 && p.MT == g16r_mt(1, 2)) return launch_block16r<1, g16r_mt(1, 2), 2>(a, st);
    if (p.NT == 2 && p.MT == g16r_mt(2, 2)) return launch_block16r<2, g16r_mt(2, 2), 2>(a, st);
    if (p.NT == 3 && p.MT == g16r_mt(3, 2)) return launch_block16r<3, g16r_mt(3, 2), 2>(a, st);
  }""", ""),
    ("""  HONK_CASE(1, 2) HONK_CASE(1, 3) HONK_CASE(1, 4) HONK_CASE(1, 5) HONK_CASE(1, 6)
  HONK_CASE(2, 2) HONK_CASE(2, 3) HONK_CASE(2, 4) HONK_CASE(2, 5) HONK_CASE(2, 6)
  HONK_CASE(3, 2) HONK_CASE(3, 3) HONK_CASE(3, 4) HONK_CASE(3, 5)
  HONK_CASE(4, 2)""", ""),
    ("""    if (L.NT == 1) rc = launch_conv0m_nt<1, FM, ONES>(L, x, out, w0, n, st, cscale);
    else if (L.NT == 2) rc = launch_conv0m_nt<2, FM, ONES>(L, x, out, w0, n, st, cscale);
    else if (L.NT == 3)""", "    if (L.NT == 3)"),
    ("""  if constexpr (FM == 2) return launch_conv0<_Float16, false, ONES>(L, x, (_Float16*)out, w0, n, st, cscale);
  else return launch_conv0<__bf16, FM == 1, ONES>(L, x, (__bf16*)out, w0, n, st);""", "  return HONK_ERR_UNSUPPORTED;"),
    ("      rc = launch_conv0_16<0, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);\n      if (rc) return rc;\n"
     "      rc = L.NT == 3 ? launch_block16n<3>(L, R, frb, frl, chsum, n, st) : launch_block16n<2>(L, R, frb, frl, chsum, n, st);",
     "      rc = HONK_ERR_UNSUPPORTED;"),
    ("""      rc = (FM == 1) ? launch_conv0_16<1, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st)
           : (FM == 2) ? launch_conv0_16<2, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st, cscale)
                       : launch_conv0_16<0, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);""",
     """      rc = launch_conv0_16<2, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st, cscale);"""),
    ("""            if (FM == 1 && pp.ppr == 9) hipLaunchKernelGGL((block16p_kernel<3, 2, 9, 9, 1>), gd, bd, 0, st, pa);
            else if (FM == 1 && pp.ppr == 5) hipLaunchKernelGGL((block16p_kernel<3, 2, 5, 10, 1>), gd, bd, 0, st, pa);
            else if (FM == 1) hipLaunchKernelGGL((block16p_kernel<3, 2, 3, 9, 1>), gd, bd, 0, st, pa);
            else if (FM == 2 && pp.ppr == 4)""", "            if (FM == 2 && pp.ppr == 4)"),
    ("""            else if (FM == 2) hipLaunchKernelGGL((block16p_kernel<3, 1, 2, 5, 1, 2>), gd, bd, 0, st, pa);
            else if (pp.ppr == 4 && pp.ns == 2) hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 2>), gd, bd, 0, st, pa);
            else if (pp.ppr == 4) hipLaunchKernelGGL((block16p_kernel<3, 1, 4, 4, 1>), gd, bd, 0, st, pa);
            else hipLaunchKernelGGL((block16p_kernel<3, 1, 2, 5, 1>), gd, bd, 0, st, pa);""", ""),
    ("""            if (FM == 1) hipLaunchKernelGGL((block16l_kernel<3, 2, 9, 9, 2>), gd, bd, 0, st, pa);
            else if (FM == 2) hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2, 2>), gd, bd, 0, st, pa);
            else hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2>), gd, bd, 0, st, pa);""",
     """            if (FM == 2) hipLaunchKernelGGL((block16l_kernel<3, 1, 4, 4, 2, 2>), gd, bd, 0, st, pa);"""),
    ("""      rc = (SP == 2) ? launch_conv0_16<1, false>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st)
                     : launch_conv0_16<0, false>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);""",
     "      rc = HONK_ERR_UNSUPPORTED;"),
    ("    rc = launch_conv0(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);", "    rc = HONK_ERR_UNSUPPORTED;"),
]

# ---- variants: patches to res_bf16p.inc ---------------------------------------------
EPI = ("        if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S) epi_step(",
       f"        if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S) if ({NEVER}) epi_step(")
RES = ("      if constexpr (ISB && S == 0) res_loads(rvs[PAR], cur.pix);",
       f"      if constexpr (ISB && S == 0) if ({NEVER}) res_loads(rvs[PAR], cur.pix);")
DMA = ("        dma(widx ? roff[rb] : roff[ra],", f"        if ({NEVER}) dma(widx ? roff[rb] : roff[ra],")
BAR = ("      __builtin_amdgcn_s_barrier();\n      asm volatile(\"\" ::: \"memory\");\n      if constexpr (TBL) {",
       f"      if ({NEVER}) __builtin_amdgcn_s_barrier();\n      asm volatile(\"\" ::: \"memory\");\n      if constexpr (TBL) {{")
WALK = ("      if constexpr (S == KW) walk_adv(wk);", f"      if constexpr (S == KW) if ({NEVER}) walk_adv(wk);")
GEO = ("      if constexpr (S == KG) nxt = geo(wk);", f"      if constexpr (S == KG) if ({NEVER}) nxt = geo(wk);")
MAXR = ("common.h", "__device__ __forceinline__ float relu_keepnan(float x) { return x <= 0.f ? 0.f : x; }",
        "__device__ __forceinline__ float relu_keepnan(float x) { return __builtin_elementwise_maximum(x, 0.f); }")
PD6 = ("  constexpr int KSA = G::KSA, PD = G::PD, CB = G::CB, CP = G::CP, P = Q::P;",
       "  constexpr int KSA = G::KSA, PD = 6, CB = G::CB, CP = G::CP, P = Q::P;")
PD3 = ("  constexpr int KSA = G::KSA, PD = G::PD, CB = G::CB, CP = G::CP, P = Q::P;",
       "  constexpr int KSA = G::KSA, PD = 3, CB = G::CB, CP = G::CP, P = Q::P;")
PIN56 = ("          if ((pt * KSA + s) * NT + n < (NS * WPS > 4 ? 33 : 64)) asm volatile",
         "          if ((pt * KSA + s) * NT + n < (NS * WPS > 4 ? 33 : 56)) asm volatile")
PIN60 = ("          if ((pt * KSA + s) * NT + n < (NS * WPS > 4 ? 33 : 64)) asm volatile",
         "          if ((pt * KSA + s) * NT + n < (NS * WPS > 4 ? 33 : 60)) asm volatile")
# compile-time removals (no per-k-step branches left behind; an empty asm keeps the
# accumulators -- hence the MFMAs -- alive at no cost)
EPI2 = ("epi_step(rolec, ec, std::integral_constant<int, 1 - PAR>{});",
        "sink(std::integral_constant<int, 1 - PAR>{}, ec);")
EPI2b = ("  auto res_loads = [&](uint4 (&rvn)[G::NRF][SP], unsigned po) {",
         "  auto sink = [&](auto pendc, auto ec) {\n"
         "    constexpr int PQ = decltype(pendc)::value, E = decltype(ec)::value;\n"
         "    if constexpr (E < NT) { const f32x4 t = accs[PQ][E]; asm volatile(\"\" :: \"a\"(t)); }\n"
         "  };\n"
         "  auto res_loads = [&](uint4 (&rvn)[G::NRF][SP], unsigned po) {")
RES2 = ("      if constexpr (ISB && S == 0) res_loads(rvs[PAR], cur.pix);", "")
DMA2 = ("""        dma(widx ? roff[rb] : roff[ra], widx ? rslot[rb] : rslot[ra], std::integral_constant<int, pa>{},
            std::integral_constant<int, pb>{}, rr < nnew);""", "        (void)rr;")
WALK2 = ("      if constexpr (S == KW) walk_adv(wk);", "")
GEO2 = ("      if constexpr (S == KG) nxt = geo(wk);", "      if constexpr (S == KG) nxt = cur;")
NOCOK = ("    const bool cok[3] = {k.w >= sc, true, k.w + sc < W};", "    const bool cok[3] = {true, true, true};")
NOROK = ("    const bool rok[3] = {valid && k.j >= sr, valid, valid && k.j + sr < k.n};",
         "    const bool rok[3] = {valid, valid, valid};")
def kwkg(kw, kg):
    return [("  constexpr int KW = 4;                  // k-step of the walk's advance",
             f"  constexpr int KW = {kw};"),
            ("  constexpr int KG = KSA - 1 - PD - 1;   // k-step of the next m-tile's geometry",
             f"  constexpr int KG = {kg};")]
BALON = ("  constexpr bool BAL = false;", "  constexpr bool BAL = true;")
NOEPIA = ("          if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S) epi_step(rolec, ec, std::integral_constant<int, 1 - PAR>{});",
          "          if constexpr ((KE + E < KSA ? KE + E : KSA - 1) == S && decltype(rolec)::value) epi_step(rolec, ec, std::integral_constant<int, 1 - PAR>{});")
WALKT = ("        if constexpr (S == KW) walk_adv_t(wk);", "")
GEOT = ("        if constexpr (S == KG) nxt = geo_t(wk);", "        if constexpr (S == KG) nxt = cur;")
# memory-latency probes: the same accesses at L2-resident addresses / without the DMA wait
RESL2 = ("      if constexpr (ISB && S == 0) res_loads(rvs[PAR], cur.pix);",
         "      if constexpr (ISB && S == 0) res_loads(rvs[PAR], cur.pix & 0xFFFFu);")
DMAL2 = ("16, (v == 0xffffu || !ok) ? 0xF0000000u : off + v, 0, 0, 0);",
         "16, (v == 0xffffu || !ok) ? 0xF0000000u : (off & 0xFFFFu) + v, 0, 0, 0);")
NOWAIT = ("      if constexpr (!ISB) wait_vmcnt<0>();\n      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)\n      __builtin_amdgcn_s_barrier();",
          "      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)\n      __builtin_amdgcn_s_barrier();")
NOSTORE = ("            __builtin_amdgcn_raw_buffer_store_b128(v4, rrs, ppix + 16 * g,",
           f"            if ({NEVER}) __builtin_amdgcn_raw_buffer_store_b128(v4, rrs, ppix + 16 * g,")
# in-kernel stamps (diagnostic build): per wave, cycles in the step loop, at the DMA wait,
# at the barrier; read back through honk_dbg_read
STAMP = [
    ("  float* chsum;         // last-layer mode: [nclips][2][CP] channel sums of relu(A's output)\n};",
     "  float* chsum;         // last-layer mode: [nclips][2][CP] channel sums of relu(A's output)\n  unsigned long long* dbg;\n};"),
    ("    for (int k = 0; k < nsteps; ++k) {\n      // step barrier",
     "    unsigned long long t_all = __builtin_amdgcn_s_memtime(), t_vm = 0, t_bar = 0;\n    for (int k = 0; k < nsteps; ++k) {\n      // step barrier"),
    ("      asm volatile(\"\" ::: \"memory\");\n      if constexpr (!ISB) wait_vmcnt<0>();",
     "      asm volatile(\"\" ::: \"memory\");\n      const unsigned long long ta = __builtin_amdgcn_s_memtime();\n      if constexpr (!ISB) wait_vmcnt<0>();"),
    ("      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)\n      __builtin_amdgcn_s_barrier();\n      asm volatile(\"\" ::: \"memory\");\n      if constexpr (TBL) {",
     "      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)\n      const unsigned long long tb = __builtin_amdgcn_s_memtime();\n      __builtin_amdgcn_s_barrier();\n      const unsigned long long tc = __builtin_amdgcn_s_memtime();\n      t_vm += tb - ta;\n      t_bar += tc - tb;\n      asm volatile(\"\" ::: \"memory\");\n      if constexpr (TBL) {"),
    ("    wait_vmcnt<0>();\n    static_for<ELAST + 1>([&](auto ec) { epi_step(rolec, ec, std::integral_constant<int, 1>{}); });",
     "    wait_vmcnt<0>();\n    static_for<ELAST + 1>([&](auto ec) { epi_step(rolec, ec, std::integral_constant<int, 1>{}); });\n"
     "    t_all = __builtin_amdgcn_s_memtime() - t_all;\n"
     "    if (!LM && a.dbg && lane == 0) {\n"
     "      unsigned long long* o = a.dbg + ((size_t)blockIdx.x * 8 + wave) * 4;\n"
     "      o[0] = t_all; o[1] = t_vm; o[2] = t_bar; o[3] = (unsigned long long)nsteps;\n    }"),
    ("res.hip", "            pa.chsum = nullptr;", "            pa.chsum = nullptr;\n            pa.dbg = honk_dbg_buf();"),
    ("res.hip", "            pa.chsum = chsum;", "            pa.chsum = chsum;\n            pa.dbg = nullptr;"),
    ("res.hip", "struct PairPlan {", "static unsigned long long* honk_dbg_buf() {\n  static unsigned long long* b = nullptr;\n"
     "  if (!b) { (void)hipMalloc(&b, 1 << 20); (void)hipMemset(b, 0, 1 << 20); }\n  return b;\n}\nstruct PairPlan {"),
    ("res.hip", "extern \"C\" {", "extern \"C\" {\n"
     "int honk_dbg_read(unsigned long long* h, int n) { (void)hipDeviceSynchronize(); return (int)hipMemcpy(h, honk::res::honk_dbg_buf(), n * 8, hipMemcpyDeviceToHost); }"),
]
VARIANTS_OLD3 = []
VARIANTS = {
    "stamp": STAMP,
    "stampsametq": STAMP + [("        if constexpr (S == KG) nxt = geo_t(wk);",
                 "        if constexpr (S == KG) { const MG g2 = geo_t(wk); nxt = cur; nxt.pix = g2.pix; nxt.lo = g2.lo; }")],
    "stampdmaA": STAMP + [("  constexpr bool DMAB = !LM;", "  constexpr bool DMAB = false;")],
    "stampnogeo": STAMP + [WALKT, GEOT],
    "stampnodma": STAMP + [DMA2],
    "stampmfma": STAMP + [EPI2b, EPI2, RES2, DMA2, WALKT, GEOT],
    "nogeoT": [WALKT, GEOT],
    "bal": [BALON],
    "padall": [("  constexpr bool PADC = TBL && LM;", "  constexpr bool PADC = TBL;"),
               ("res.hip", "  if (FM == 2 && padcols) {", "  if (FM == 2) {")],
    "padall1k": [("  constexpr bool PADC = TBL && LM;", "  constexpr bool PADC = TBL;"),
                 ("res.hip", "  if (FM == 2 && padcols) {", "  if (FM == 2) {"),
                 ("res.hip", "    pp.padb = (int)((sc * PXB + 255) / 256 * 256);", "    pp.padb = (int)((sc * PXB + 1023) / 1024 * 1024);"),
                 ("res.hip", "    pp.slotb = (int)((pp.padb + right + 255) / 256 * 256);", "    pp.slotb = (int)((pp.padb + right + 1023) / 1024 * 1024);")],
    # which part of the geometry costs: the table read, the tap addresses, the pixel addresses
    "gnoread": [("    k.e = *(const u32x4*)e;\n    k.lo = *(const int*)(e + 16);",
                 "    k.e = u32x4{(unsigned)(k.r & 1) * 4096u + (unsigned)ringA, (unsigned)ringA + 4096u, (unsigned)ringA + 8192u, (unsigned)(k.r * 3840)};\n    k.lo = ringB + (k.r & 3) * 4096;")],
    "gnozrow": [("      if (j >= sr) rb0 = ring + ((r - sr) % nr) * a.slotb + padb;\n      if (j + sr < n) rb2 = ring + ((r + sr) % nr) * a.slotb + padb;",
                 "      rb0 = ring + ((r + nr - sr) % nr) * a.slotb + padb;\n      rb2 = ring + ((r + sr) % nr) * a.slotb + padb;")],
    "gnozero": [("      if (j >= sr) rb0 = ring + ((r - sr) % nr) * a.slotb + padb;\n      if (j + sr < n) rb2 = ring + ((r + sr) % nr) * a.slotb + padb;",
                 "      rb0 = ring + ((r + nr - sr) % nr) * a.slotb + padb;\n      rb2 = ring + ((r + sr) % nr) * a.slotb + padb;"),
                ("      for (int dx = 0; dx < 3; ++dx) m.tq[DY * 3 + dx] = ok[dx] ? rb + tk[DY * 3 + dx] : zg0;",
                 "      for (int dx = 0; dx < 3; ++dx) m.tq[DY * 3 + dx] = rb + tk[DY * 3 + dx] - (ok[dx] ? 0 : (dx - 1) * scb);")],
    "kw1kg3": kwkg(1, 3),
    "kw1kg2": kwkg(1, 2),
    "kw0kg2": kwkg(0, 2),
    "gsametq": [("        if constexpr (S == KG) nxt = geo_t(wk);",
                 "        if constexpr (S == KG) { const MG g2 = geo_t(wk); nxt = cur; nxt.pix = g2.pix; nxt.lo = g2.lo; }")],
    "gsamepix": [("        if constexpr (S == KG) nxt = geo_t(wk);",
                  "        if constexpr (S == KG) { const MG g2 = geo_t(wk); nxt = g2; nxt.pix = cur.pix; nxt.lo = cur.lo; }")],
    "dsp2": [("  constexpr int DSP = 1;", "  constexpr int DSP = 2;")],
    "dsp3": [("  constexpr int DSP = 1;", "  constexpr int DSP = 3;")],
    "dsp4": [("  constexpr int DSP = 1;", "  constexpr int DSP = 4;")],
    "pin60": [PIN60],
    "pin56": [PIN56],
    "pin48": [("          if ((pt * KSA + s) * NT + n < (NS * WPS > 4 ? 33 : 64)) asm volatile",
               "          if ((pt * KSA + s) * NT + n < (NS * WPS > 4 ? 33 : 48)) asm volatile")],
    "dmaA": [("  constexpr bool DMAB = !LM;", "  constexpr bool DMAB = false;")],
    "pd1": [("  constexpr int PD = (FM == 2 && KSA % 7 == 0) ? 6 : G::PD;", "  constexpr int PD = G::PD;")],
    "noB": [("    if (role == 0) run_role(std::integral_constant<bool, false>{});\n    else run_role(std::integral_constant<bool, true>{});",
             "    if (role == 0) run_role(std::integral_constant<bool, false>{});\n    else for (int k = 0; k < nsteps; ++k) __builtin_amdgcn_s_barrier();")],
    "noA": [("    if (role == 0) run_role(std::integral_constant<bool, false>{});\n    else run_role(std::integral_constant<bool, true>{});",
             "    if (role == 0) { for (int k = 0; k < nsteps; ++k) __builtin_amdgcn_s_barrier(); }\n    else run_role(std::integral_constant<bool, true>{});")],
    "nomix": [("res_bf16w.inc", "  if constexpr (FM == 2) {\n    float out;", "  if constexpr (FM == 22) {\n    float out;")],
    "balpd6": [BALON, PD6],
    "nodma": [DMA2],
    "nobar": [BAR],
    "noslp": [("CFLAGS", "-fno-slp-vectorize", "")],
    "noepiA": [NOEPIA],
    "mfmaT": [EPI2b, EPI2, RES2, DMA2, BAR, WALKT, GEOT],
    "resl2": [RESL2],
    "dmal2": [DMAL2],
    "nowait": [NOWAIT],
    "nostore": [NOSTORE],
    "memL2": [RESL2, DMAL2, NOSTORE],
    "base": [],
    "mfma": [EPI, RES, DMA, BAR, WALK, GEO],   # MFMAs + their operand reads only
    "noepi": [EPI, RES],
    "nogeo": [WALK, GEO],
    "nobar": [BAR],
    "nodma": [DMA],
    "max": [MAXR],
    "pd6": [PD6],
    "pd6mfma": [PD6, EPI, RES, DMA, BAR, WALK, GEO],
    "pin56": [PIN56],
    "pin60": [PIN60],
    "maxpd6": [MAXR, PD6],
    "mfma2": [EPI2b, EPI2, RES2, DMA2, BAR, WALK2, GEO2],
    "mfma2pd6": [PD6, EPI2b, EPI2, RES2, DMA2, BAR, WALK2, GEO2],
    "noepi2": [EPI2b, EPI2, RES2],
    "nogeo2": [WALK2, GEO2],
    "nocok": [NOCOK],
    "novalid": [NOCOK, NOROK],
    "oldsel": [("        return (tq[tB] & hi2) | (tq[tA] & ~hi2);",
                "        if constexpr (TBL) return (tq[tB] & hi2) | (tq[tA] & ~hi2);\n        else return tq[tA] + ((tq[tB] - tq[tA]) & hi2);")],
    "oldsel26": [("        return (tq[tB] & hi2) | (tq[tA] & ~hi2);",
                "        if constexpr (TBL) return (tq[tB] & hi2) | (tq[tA] & ~hi2);\n        else return tq[tA] + ((tq[tB] - tq[tA]) & hi2);"),
                 ("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 26 : 64)")],
    "oldrelu": [("common.h", "{ return __builtin_elementwise_maximum(x, 0.f); }", "{ return x <= 0.f ? 0.f : x; }")],
    "oldact": [("res_bf16w.inc", """          float r = act_dec<FM>(rv[f][0][e >> 1], e);
          if constexpr (SP == 2) r += act_dec<FM>(rv[f][1][e >> 1], e);""", """          float r = 0.f;
#pragma unroll
          for (int pt = 0; pt < SP; ++pt) r += act_dec<FM>(rv[f][pt][e >> 1], e);""")],
    "old3": VARIANTS_OLD3,
    "pin24": [("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 24 : 64)")],
    "pin28": [("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 28 : 64)")],
    "pin26": [("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 26 : 64)")],
    "pin30": [("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 30 : 64)")],
    "pin36": [("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 36 : 64)")],
    "pin40": [("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 40 : 64)")],
    "pin20": [("(NS * WPS > 4 ? 33 : 64)", "(NS * WPS > 4 ? 20 : 64)")],
    "kg6": kwkg(3, 6),
    "kg3": kwkg(1, 3),
    "kg8": kwkg(4, 8),
}


def build(name, patches=None):
    if name == "old3":
        patches = VARIANTS["oldrelu"] + VARIANTS["oldact"] + VARIANTS["oldsel"]
    d = os.path.join(OUT, name)
    src = os.path.join(d, "src")
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    shutil.copytree(os.path.join(ROOT, "honk_amd", "csrc"), os.path.join(src, "honk_amd", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(src, "include"))
    csrc = os.path.join(src, "honk_amd", "csrc")
    f = os.path.join(csrc, "res.hip")
    s = open(f).read()
    for a, b in (REDUCE if not os.environ.get("PAIR_FULL") else []):
        assert a in s, ("reduce", a[:80])
        s = s.replace(a, b)
    open(f, "w").write(s)
    cflags = []
    for pt in (patches if patches is not None else VARIANTS[name]):
        fn, a, b = pt if len(pt) == 3 else ("res_bf16p.inc",) + tuple(pt)
        if fn == "CFLAGS":
            cflags.append(a)
            continue
        f = os.path.join(csrc, fn)
        s = open(f).read()
        assert a in s, (name, fn, a[:80])
        s = s.replace(a, b)
        open(f, "w").write(s)
    sys.path.insert(0, ROOT)
    from honk_amd.build import FLAGS
    cc = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-function",
          "-save-temps=obj", "-I", os.path.join(src, "include")]
    objs = []  # res.hip and res_vf.hip (the f16x2 pair / last layer, with their own flags)
    procs = []
    for tu in ("res.hip", "res_vf.hip"):
        objs.append(os.path.join(d, tu.replace(".hip", ".o")))
        procs.append(subprocess.Popen(cc + FLAGS.get(tu, []) + cflags + ["-c", os.path.join(csrc, tu), "-o", objs[-1]]))
    assert all(p.wait() == 0 for p in procs), name
    bd = os.path.join(ROOT, "honk_amd", "_build")
    others = [os.path.join(bd, x + ".o") for x in ("runtime", "cnn", "train", "mfcc", "head", "augment")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(d, "libhonk_hip.so")] + objs + others, check=True)
    shutil.rmtree(src)
    for t in glob.glob(os.path.join(d, "*")):
        if not t.endswith((".so", "-gfx950.s")):
            os.remove(t)
    return name


RUN = r'''
import os, sys, torch
sys.path.insert(0, os.getcwd())
from honk_amd import model as hm
torch.manual_seed(0)
m = hm.find_model("res15")(dict(hm.find_config("res15"))).eval().cuda()
m.honk_precision, m.honk_reroute = os.environ.get("PAIR_PREC", "f16x2"), False
x = torch.randn(8192, 101, 40, device="cuda")
with torch.no_grad():
    for _ in range(3):
        m(x)
torch.cuda.synchronize()
'''


def time_variants(names):
    import csv
    for name in names:
        lib = os.path.join(OUT, name, "libhonk_hip.so")
        od = os.path.join(ROOT, "gpurun_out", "pair", name)
        os.makedirs(od, exist_ok=True)
        env = dict(os.environ, HONK_LIB=lib)
        r = subprocess.run(["timeout", "-k", "10", "120", "rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", od, "-o", "run",
                            "--", sys.executable, "-c", RUN], env=env, capture_output=True, text=True)
        if r.returncode != 0:
            print(name, "FAILED", r.returncode, r.stderr[-1500:], flush=True)
            sys.exit(r.returncode)
        stats = glob.glob(os.path.join(od, "**", "*kernel_stats.csv"), recursive=True)
        row = {}
        with open(stats[0]) as fh:
            for rec in csv.DictReader(fh):
                k = rec["Name"]
                for tag in ("block16p_kernel", "block16l_kernel", "conv0m_kernel"):
                    if tag in k:
                        row[tag] = round(float(rec["AverageNs"]) / 1e3, 1)
        print(f"{name:12s} " + "  ".join(f"{k} {v} us" for k, v in sorted(row.items())), flush=True)


RUNSTAMP = RUN + r'''
import ctypes, numpy as np
lib = ctypes.CDLL(os.environ["HONK_LIB"])
buf = np.zeros(256 * 8 * 4, dtype=np.uint64)
lib.honk_dbg_read(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
b = buf.reshape(256, 8, 4).astype(np.float64)
for role, ws in (("A", [0, 1]), ("B", [2, 3])):
    t = b[:, ws, :]
    print(f"{role}: loop {np.median(t[..., 0]) / 1e3:.1f}K cyc  dma-wait {np.median(t[..., 1]) / 1e3:.1f}K  barrier {np.median(t[..., 2]) / 1e3:.1f}K"
          f"  steps {np.median(t[..., 3]):.0f}  per step {np.median(t[..., 0] / t[..., 3]):.0f} cyc"
          f" (wait {np.median(t[..., 1] / t[..., 3]):.0f}, bar {np.median(t[..., 2] / t[..., 3]):.0f})")
'''


def stamp_run(name):
    lib = os.path.join(OUT, name, "libhonk_hip.so")
    env = dict(os.environ, HONK_LIB=lib)
    r = subprocess.run(["timeout", "-k", "10", "120", sys.executable, "-c", RUNSTAMP], env=env, capture_output=True, text=True)
    print(name, r.returncode, r.stdout[-3000:], r.stderr[-2000:] if r.returncode else "", flush=True)


PMC = "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"


def pmc_variants(names):
    """one --pmc pass per variant (kernel-trace only beside it): per-launch means of the pair kernel"""
    import csv
    from collections import defaultdict
    for name in names:
        lib = os.path.join(OUT, name, "libhonk_hip.so")
        od = os.path.join(ROOT, "gpurun_out", "pairpmc", name)
        os.makedirs(od, exist_ok=True)
        env = dict(os.environ, HONK_LIB=lib)
        r = subprocess.run(["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc"] + PMC.split() +
                           ["--output-format", "csv", "-d", od, "-o", "run", "--", sys.executable, "-c", RUN],
                           env=env, capture_output=True, text=True)
        if r.returncode != 0:
            print(name, "FAILED", r.returncode, r.stderr[-1500:], flush=True)
            sys.exit(r.returncode)
        f = glob.glob(os.path.join(od, "**", "*counter_collection.csv"), recursive=True)[0]
        acc = defaultdict(lambda: defaultdict(list))
        with open(f) as fh:
            for rec in csv.DictReader(fh):
                for tag in ("block16p_kernel", "block16l_kernel"):
                    if tag in rec["Kernel_Name"]:
                        acc[tag][rec["Counter_Name"]].append(float(rec["Counter_Value"]))
        for tag, cs in acc.items():
            m = {k: sum(v) / len(v) for k, v in cs.items()}
            print(f"{name:10s} {tag}: " + " ".join(f"{k.replace('SQ_', '')}={v:.4g}" for k, v in sorted(m.items())), flush=True)


if __name__ == "__main__":
    cmd, names = sys.argv[1], sys.argv[2:] or list(VARIANTS)
    if cmd == "build":
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(min(len(names), 6)) as ex:
            for n in ex.map(build, names):
                print("built", n, flush=True)
    elif cmd == "stamp":
        for n in names:
            stamp_run(n)
    elif cmd == "pmc":
        pmc_variants(names)
    else:
        time_variants(names)

"""The register-spill guard: tools/check_spills.py over the device
assembly honk_amd.build keeps (-save-temps) -- no kernel of libhonk_hip.so restores a
register tuple in part before an instruction reads it whole (the LLVM partial-spill
miscompile behind round 4's wrong bf16 logits), and the detector fires on that shape."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_spills as cs  # noqa: E402

SPLIT = """
_Z3fooi:
	scratch_store_dwordx3 off, v[10:12], off offset:16 ; 12-byte Folded Spill
	scratch_load_dwordx3 v[20:22], off, off offset:16 ; 12-byte Folded Reload
	v_mfma_f32_16x16x32_bf16 v[0:3], v[20:23], v[4:7], v[0:3]
.Lfunc_end0:
_Z3bari:
	scratch_store_dwordx4 off, v[10:13], off ; 16-byte Folded Spill
	scratch_load_dwordx4 v[20:23], off, off ; 16-byte Folded Reload
	v_mfma_f32_16x16x32_bf16 v[0:3], v[20:23], v[4:7], v[0:3]
.Lfunc_end1:
_Z3bazi:
	scratch_store_dwordx2 off, v[14:15], off offset:32 ; 8-byte Folded Spill
	scratch_load_dwordx2 v[16:17], off, off offset:32 ; 8-byte Folded Reload
	v_mad_u64_u32 v[16:17], s[14:15], v14, s21, v[16:17]
	v_mov_b32_e32 v40, v2 ; Reload Reuse
.Lfunc_end2:
"""


def test_detector_tells_split_from_whole():
    got = {k: st for k, st, _ in cs.scan_asm(SPLIT)}
    assert got["foo(int)"] == "SPLIT"        # a 12-byte reload feeding a 16-byte MFMA operand
    assert got["bar(int)"] == "spill"        # a whole 16-byte fragment
    assert got["baz(int)"] == "SPLIT"        # a Reload Reuse annotation


# the reload's first reader reads a subset (v21), a later MFMA reads past it;
# a reload at the bottom of a loop whose wide reader sits at the loop head; the
# 8/12-byte-spill backstop; and a reloaded register rewritten before any wide read (clean)
SPLIT2 = """
_Z4sub1i:
	scratch_load_dwordx3 v[20:22], off, off offset:16 ; 12-byte Folded Reload
	v_mov_b32_e32 v40, v21
	v_mfma_f32_16x16x32_bf16 v[0:3], v[20:23], v[4:7], v[0:3]
.Lfunc_end0:
_Z4loopi:
.LBB1_1:
	v_mfma_f32_16x16x32_bf16 v[0:3], v[20:23], v[4:7], v[0:3]
	s_add_u32 s4, s4, 1
	scratch_load_dwordx3 v[20:22], off, off offset:16 ; 12-byte Folded Reload
	s_cbranch_scc1 .LBB1_1
	s_endpgm
.Lfunc_end1:
_Z4backi:
	scratch_store_dwordx3 off, v[30:32], off offset:48 ; 12-byte Folded Spill
	v_mfma_f32_16x16x32_f16 v[0:3], v[30:33], v[4:7], v[0:3]
.Lfunc_end2:
_Z4killi:
	scratch_load_dwordx4 v[20:23], off, off ; 16-byte Folded Reload
	v_mov_b32_e32 v40, v21
	v_mov_b32_e32 v20, 0
	v_mov_b32_e32 v21, 0
	v_mov_b32_e32 v22, 0
	v_mov_b32_e32 v23, 0
	v_mfma_f32_16x16x32_bf16 v[0:3], v[18:21], v[4:7], v[0:3]
.Lfunc_end3:
"""


def test_detector_follows_reads_past_the_first_and_around_loops():
    got = {k: (st, d) for k, st, d in cs.scan_asm(SPLIT2)}
    assert got["sub1(int)"][0] == "SPLIT", got      # a subset read first, then the wide one
    assert got["loop(int)"][0] == "SPLIT", got      # the wide reader is at the loop head
    assert got["back(int)"][0] == "SPLIT", got      # 12-byte spill, registers read 16 wide
    assert got.get("kill(int)", ("clean",))[0] != "SPLIT", got  # rewritten before the wide read


def test_library_has_no_split_spills():
    from honk_amd import build
    build.build()   # incremental; keeps the device assembly of every csrc/*.hip
    files = cs.default_files()
    srcs = [f for f in build.SOURCES if f.endswith(".hip")]
    assert len(files) >= len(srcs), (files, srcs)
    assert cs.check_files(files, verbose=True) == []

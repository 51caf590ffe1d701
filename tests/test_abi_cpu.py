"""CPU-side checks of the drop-in boundary: libhvx.so loads and exports every symbol that
include/hvx.h declares; the ABI struct mirrors match the C layouts; no compute calls."""
import ctypes
import os
import re
import subprocess

import numpy as np

from video_codecs_amd import _abi, hvx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "hvx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void \*|const char \*)\s*(hvx_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    L = hvx.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert L.hvx_version() == 1


def test_no_gpu_is_a_loud_error():
    import torch
    if torch.cuda.is_available():
        return
    p = ctypes.c_void_p()
    rc = hvx.lib().hvx_create(0, ctypes.byref(p))
    assert rc != 0
    try:
        hvx.context()
    except hvx.HvxError:
        pass
    else:
        raise AssertionError("hvx.context() must raise without a GPU")


def test_struct_layouts_match_c():
    # compile a tiny C program printing sizeof/offsetof of the ABI structs
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "hvx.h"
int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(hvx_tu_desc), offsetof(hvx_tu_desc, lambda),
 sizeof(hvx_estbits), sizeof(hvx_me_job), sizeof(hvx_me_result), sizeof(hvx_dist_job), sizeof(hvx_interp_job),
 sizeof(hvx_ssim_job), sizeof(hvx_stvssim_job), offsetof(hvx_me_job, lambda_motion)); return 0;}
"""
    tmp = "/tmp/hvx_layout_check"
    with open(tmp + ".c", "w") as f:
        f.write(prog)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp])
    vals = [int(x) for x in subprocess.check_output([tmp]).split()]
    assert vals == [_abi.TU_DESC.itemsize, _abi.TU_DESC.fields["lambda"][1], _abi.ESTBITS_INTS * 4,
                    _abi.ME_JOB.itemsize, _abi.ME_RESULT.itemsize, hvx.DIST_JOB.itemsize, hvx.INTERP_JOB.itemsize,
                    hvx.SSIM_JOB.itemsize, hvx.STVSSIM_JOB.itemsize, _abi.ME_JOB.fields["lambda_motion"][1]]


def test_sao_decide_job_layout_matches_c():
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "hvx.h"
int main(){printf("%zu %zu %zu %zu %zu\n", sizeof(hvx_sao_decide_job), offsetof(hvx_sao_decide_job, sao_states),
 offsetof(hvx_sao_decide_job, lambda), offsetof(hvx_sao_decide_job, stats), offsetof(hvx_sao_decide_job, total_cost)); return 0;}
"""
    tmp = "/tmp/hvx_saodec_layout"
    with open(tmp + ".c", "w") as f:
        f.write(prog)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp])
    vals = [int(x) for x in subprocess.check_output([tmp]).split()]
    J = _abi.SAO_DECIDE_JOB
    assert vals == [J.itemsize, J.fields["sao_states"][1], J.fields["lambda"][1], J.fields["stats"][1], J.fields["total_cost"][1]]


def test_golden_estbits_layout():
    from tests import golden_cases as gc
    g = gc.load("tu_ldp.bin")
    assert g["fwd_estbits"].shape[1] == _abi.ESTBITS_INTS


def test_estbits_update_host_golden():
    # the library's host form of TEncSbac::estBit (product code, no device) vs the reference
    from tests import golden_cases as gc
    g = gc.load("estbit.bin")
    meta, states, rice, before, after, eb = g["meta"], g["states"], g["rice"], g["before"], g["after"], g["entropy_bits"]
    for i in range(meta.shape[0]):
        w, h, ch = (int(x) for x in meta[i, :3])
        got = hvx.estbits_update(states[i], eb, rice[i], w, h, ch, before[i])
        np.testing.assert_array_equal(got, after[i], err_msg=f"record {i}")
    # invalid geometry is an error, not a silent result
    import pytest
    with pytest.raises(hvx.HvxError):
        hvx.estbits_update(states[0], eb, rice[0], 64, 64, 0, before[0])


def test_intra_struct_layouts_match_c():
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "hvx.h"
int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(hvx_intra_job), offsetof(hvx_intra_job, avail),
 offsetof(hvx_intra_job, ctx_state), offsetof(hvx_intra_job, sqrt_lambda), sizeof(hvx_intra_search_result),
 offsetof(hvx_intra_search_result, satd), offsetof(hvx_intra_search_result, mode_bits),
 offsetof(hvx_intra_search_result, n_cand), offsetof(hvx_intra_search_result, cand)); return 0;}
"""
    tmp = "/tmp/hvx_intra_layout_check"
    with open(tmp + ".c", "w") as f:
        f.write(prog)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp])
    vals = [int(x) for x in subprocess.check_output([tmp]).split()]
    J, R = _abi.INTRA_JOB, _abi.INTRA_RESULT
    assert vals == [J.itemsize, J.fields["avail"][1], J.fields["ctx_state"][1], J.fields["sqrt_lambda"][1], R.itemsize,
                    R.fields["satd"][1], R.fields["mode_bits"][1], R.fields["n_cand"][1], R.fields["cand"][1]]


def test_deblock_params_layout_matches_c():
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "hvx.h"
int main(){printf("%zu %zu %zu\n", sizeof(hvx_deblock_params), offsetof(hvx_deblock_params, cb_qp_offset),
 offsetof(hvx_deblock_params, flags)); return 0;}
"""
    tmp = "/tmp/hvx_dbk_layout_check"
    with open(tmp + ".c", "w") as f:
        f.write(prog)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp])
    vals = [int(x) for x in subprocess.check_output([tmp]).split()]
    D = _abi.DEBLOCK_PARAMS
    assert vals == [D.itemsize, D.fields["cb_qp_offset"][1], D.fields["flags"][1]]


def test_oracle_deblock_random_smoke():
    # the random-map recipe of the GPU test runs on the oracle alone (CPU): filters fire, borders fixed
    import numpy as np
    import oracle
    rng = np.random.default_rng(1)
    ramp = np.add.outer(np.arange(64), np.arange(64)) // 3
    y = (ramp + 6 * ((np.arange(64)[None, :] // 8) % 2) + 6 * ((np.arange(64)[:, None] // 8) % 2)).astype(np.uint8)
    cb, cr = y[::2, ::2].copy(), y[::2, ::2].copy()
    bv = np.zeros((16, 16), np.uint8); bv[:, 2::2] = 2
    bh = np.zeros((16, 16), np.uint8); bh[2::2, :] = 1
    qp = np.full((16, 16), 37, np.int8)
    out = oracle.deblock(y, cb, cr, bv.ravel(), bh.ravel(), qp.ravel(), _abi.deblock_params(64, 64))
    assert (out[0] != y).any() and (out[1] != cb).any()


def test_lambda_ssim_matches_stvssim():
    # the product-side SSIM-RDO lambda (video_codecs_amd/_abi.py) is the oracle's lambda_2 /
    # adjust_lambda (pinned to stvssim.c by tests/golden/ssim.bin)
    import oracle
    for qp in (0, 15, 22, 27, 32, 37, 51):
        assert _abi.lambda_ssim(qp) == oracle.lambda_2(qp)
        assert abs(_abi.lambda_ssim(qp, 0.7) - oracle.adjust_lambda(oracle.lambda_2(qp), 0.7)) <= 1e-18


def test_new_entry_points_reject_bad_arguments_without_a_gpu():
    # argument validation happens before any device work: NULL context / pointers and out-of-range
    # deblocking parameters fail with HVX_E_INVALID and a message (HM-style fail-fast callers abort)
    import ctypes
    L = ctypes.CDLL(os.path.join(ROOT, "video_codecs_amd", "libhvx.so"))
    L.hvx_last_error.restype = ctypes.c_char_p
    E_INVALID = -1
    P = ctypes.c_void_p
    assert L.hvx_intra_pred_batch(P(0), P(0), 64, P(0), 1, P(0), P(0), P(0)) == E_INVALID
    assert b"hvx_intra_pred_batch" in L.hvx_last_error()
    assert L.hvx_intra_search_batch(P(0), P(0), P(0), 64, P(0), 1, P(0), P(0)) == E_INVALID
    assert L.hvx_deblock(P(0), P(0), 64, P(0), P(0), 32, P(0), P(0), P(0), P(0)) == E_INVALID
    assert b"hvx_deblock" in L.hvx_last_error()
    # the CABAC residual writer: NULL context, negative run count / capacity
    assert L.hvx_coeff_write_batch(P(0), P(0), P(0), P(0), P(0), 1, P(0), P(0), P(0), P(0), 64, P(0)) == E_INVALID
    assert b"hvx_coeff_write_batch" in L.hvx_last_error()
    assert L.hvx_coeff_write_batch(P(0), P(0), P(0), P(0), P(0), -1, P(0), P(0), P(0), P(0), 64, P(0)) == E_INVALID


def test_cabac_regs_layout_matches_c():
    # hvx_cabac_regs (hvx_types.h) = TEncBinCABAC's registers + the bin count; start() values
    from video_codecs_amd import _abi
    assert _abi.CABAC_REGS.names == ("low", "range", "bits_left", "num_buffered", "buffered_byte", "bins", "coded")
    assert [_abi.CABAC_REGS.fields[f][1] for f in _abi.CABAC_REGS.names] == [0, 4, 8, 12, 16, 20, 24]
    assert _abi.CABAC_START[:5] == (0, 510, 23, 0, 0xFF)
    src = open(os.path.join(ROOT, "include", "hvx_types.h")).read()
    assert "typedef struct hvx_cabac_regs" in src and "uint32_t buffered_byte, bins;" in src
    assert "uint32_t coded[5];\n} hvx_cabac_regs;" in src


def test_sao_layout_matches_c():
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "hvx.h"
int main(){printf("%zu %zu %zu %zu %zu\n", sizeof(hvx_sao_offset), offsetof(hvx_sao_offset, offset), sizeof(hvx_sao_ctu),
 sizeof(hvx_sao_stat), offsetof(hvx_sao_stat, count)); return 0;}
"""
    tmp = "/tmp/hvx_sao_layout_check"
    with open(tmp + ".c", "w") as f:
        f.write(prog)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp])
    vals = [int(x) for x in subprocess.check_output([tmp]).split()]
    O, S = _abi.SAO_OFFSET, _abi.SAO_STAT
    assert vals == [O.itemsize, O.fields["offset"][1], _abi.SAO_CTU.itemsize, S.itemsize, S.fields["count"][1]]


def test_sao_entry_points_reject_bad_arguments_without_a_gpu():
    # geometry / aliasing / partial-chroma checks run before any device work (the context is
    # only dereferenced at the launch, so a dummy non-NULL handle is enough here)
    import ctypes
    L = ctypes.CDLL(os.path.join(ROOT, "video_codecs_amd", "libhvx.so"))
    L.hvx_last_error.restype = ctypes.c_char_p
    E_INVALID = -1
    P = ctypes.c_void_p
    fake = ctypes.create_string_buffer(4096)
    ctx = P(ctypes.addressof(fake))
    buf = [ctypes.create_string_buffer(64) for _ in range(7)]
    a = [P(ctypes.addressof(b)) for b in buf]
    assert L.hvx_sao_stats(P(0), a[0], a[1], a[2], 64, 32, a[3], a[4], a[5], 64, 32, 64, 64, a[6]) == E_INVALID
    assert b"hvx_sao_stats" in L.hvx_last_error()
    # 60 is not a multiple of 8; a stride below the width; only one chroma plane given
    assert L.hvx_sao_stats(ctx, a[0], a[1], a[2], 64, 32, a[3], a[4], a[5], 64, 32, 60, 64, a[6]) == E_INVALID
    assert L.hvx_sao_stats(ctx, a[0], a[1], a[2], 32, 32, a[3], a[4], a[5], 64, 32, 64, 64, a[6]) == E_INVALID
    assert L.hvx_sao_stats(ctx, a[0], a[1], P(0), 64, 32, a[3], a[4], a[5], 64, 32, 64, 64, a[6]) == E_INVALID
    assert L.hvx_sao_apply(ctx, a[0], a[1], a[2], 64, 32, a[3], a[4], a[5], 64, 32, 64, 60, a[6]) == E_INVALID
    # in place is refused: edge classes must read the unmodified neighbours
    assert L.hvx_sao_apply(ctx, a[0], a[1], a[2], 64, 32, a[0], a[4], a[5], 64, 32, 64, 64, a[6]) == E_INVALID
    assert b"differ" in L.hvx_last_error()
    assert L.hvx_sao_apply(ctx, a[0], P(0), P(0), 64, 0, a[3], a[4], P(0), 64, 32, 64, 64, a[6]) == E_INVALID


def test_oracle_sao_random_smoke():
    # the random recipe of the GPU test on the oracle alone: every class occurs, OFF CTUs unchanged
    import numpy as np
    import oracle
    rng = np.random.default_rng(3)
    w, h = 200, 136
    y = np.clip(np.kron(rng.integers(0, 256, (h // 4, w // 4)), np.ones((4, 4), np.int64))
                + rng.integers(-2, 3, (h, w)), 0, 255).astype(np.uint8)
    org = np.clip(y.astype(np.int32) + rng.integers(-9, 10, y.shape), 0, 255).astype(np.uint8)
    st = oracle.sao_stats(org, y, 0)
    assert st.shape == (12, 5)
    assert (st["count"][:, :4, :5].sum(axis=0) > 0).all() and st["count"][:, 4].sum() > 0
    nctu = 12
    rows = np.zeros((nctu, 3, 6), np.int32)
    rows[:, :, 0] = -1
    rows[1, 0] = (2, 0, 3, 1, -1, -3)
    out = oracle.sao_apply(y, 0, _abi.sao_ctu_params(rows))
    changed = np.argwhere(out != y)
    assert len(changed) and changed[:, 0].max() < 64 and changed[:, 1].min() >= 64 and changed[:, 1].max() < 128


def test_hm_picture_layout_matches_header(tmp_path):
    """video_codecs_amd.hm.HmPicture (ctypes) has the size and field offsets of include/hvx_types.h's
    hvx_hm_picture as the C compiler lays it out (the device reads the struct the host writes)."""
    import ctypes
    import subprocess
    from video_codecs_amd import hm
    fields = [f[0] for f in hm.HmPicture._fields_]
    cnames = {"lambda_": "lambda"}
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "hvx_types.h"\nint main(void){printf("%zu", sizeof(hvx_hm_picture));'
                   + "".join('printf(" %%zu", offsetof(hvx_hm_picture, %s));' % cnames.get(f, f) for f in fields)
                   + "return 0;}\n")
    exe = tmp_path / "lay"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(hm.HmPicture)] + [getattr(hm.HmPicture, f).offset for f in fields]
    assert got == want


def test_hm_record_layouts_match_header(tmp_path):
    """The numpy records of the engine's and the slice writer's device structs (hm.HM_JOB, HM_CTU,
    HM_SLICE, HM_SLICE_RESULT) have the C sizes and field offsets of include/hvx_types.h."""
    import subprocess
    from video_codecs_amd import hm
    recs = {"hvx_hm_job": hm.HM_JOB, "hvx_hm_ctu": hm.HM_CTU, "hvx_hm_slice": hm.HM_SLICE,
            "hvx_hm_slice_result": hm.HM_SLICE_RESULT}
    src = tmp_path / "rec.c"
    body = ""
    for cn, dt in recs.items():
        body += 'printf("%%zu ", sizeof(%s));' % cn
        for f in dt.names:
            body += 'printf("%%zu ", offsetof(%s, %s));' % (cn, f)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "hvx_types.h"\nint main(void){' + body + "return 0;}\n")
    exe = tmp_path / "rec"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = []
    for dt in recs.values():
        want += [dt.itemsize] + [dt.fields[f][1] for f in dt.names]
    assert got == want

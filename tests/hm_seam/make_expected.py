"""Record the reference HM-16.5rc1 (CPU, oracle/_ref/TAppEncoder) bitstream/recon MD5s for the
HM seam test (tests/test_hm_seam.py).  Run here (needs the reference build)."""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import make_yuv  # noqa: E402

CASES = {  # name: (cfg, yuv kind, frames, qp[, width, height, extra encoder args])
    "intra_rand_qp32": ("intra.cfg", "random", 1, 32),
    "intra_smooth_qp22": ("intra.cfg", "smooth", 1, 22),
    "ldp_smooth_qp32": ("ldp.cfg", "smooth", 3, 32),
    "ldb_smooth_qp32": ("ldb.cfg", "smooth", 3, 32),  # B slices: bi-prediction, identical-motion shortcut
    "ldp_rand_qp32": ("ldp.cfg", "random", 2, 32),    # uniform random: long TZ raster searches
    "ra_smooth_qp27": ("ra.cfg", "smooth", 9, 27),    # GOP8 hierarchical B: future refs, bBi refinement
    "ra_texture_qp32": ("ra.cfg", "texture", 9, 32),  # textured content in motion: uni-L0 / uni-L1 / bi AMVP choices
    # BASELINE configs 2/3 size: 1080p, CTU-row slices (the throughput seam's chains; the partial
    # bottom row continues the chain of the row above)
    "ldp_smooth_1080p_qp32": ("ldp.cfg", "smooth", 2, 32, 1920, 1080, ["--SliceMode=1", "--SliceArgument=30"]),
    # the ends of the QP range on random content: levels in the thousands (escape codes, the Rice
    # parameter at its cap) and almost nothing coded; 208x120 (a partial CTU column and row)
    "ldp_rand_qp4": ("ldp.cfg", "random", 2, 4, 208, 120),
    "ldp_rand_qp51": ("ldp.cfg", "random", 2, 51, 208, 120),
    # the search parameters the engine takes from the encoder: a smaller TZ window, AMP off
    "ldp_rand_sr16_noamp_qp32": ("ldp.cfg", "random", 2, 32, 208, 120, ["--SearchRange=16", "--AMP=0"]),
    # a tool the device decision and writer do not implement (sign hiding off): both seams must fall
    # through to HM's own code and the encode stays the reference's
    "ldp_rand_nosbh_qp32": ("ldp.cfg", "random", 2, 32, 208, 120, ["--SignHideFlag=0"]),
    # camera content: the 3-frame QCIF clip the reference's JM trees ship (jm14.1/bin/foreman_part_qcif.yuv,
    # a data fixture, tests/golden/foreman_part_qcif.yuv), P and B slices
    "foreman_ldp_qp27": ("ldp.cfg", "foreman", 3, 27, 176, 144),
    "foreman_ldb_qp32": ("ldb.cfg", "foreman", 3, 32, 176, 144),
    "foreman_intra_qp22": ("intra.cfg", "foreman", 3, 22, 176, 144),
}
YUV_FRAMES = max(c[2] for c in CASES.values())
W, H = 416, 240


def case_size(case):
    c = CASES[case]
    return (c[4], c[5]) if len(c) > 4 else (W, H)


def encode(binary, case, tmp, log=None):
    """Encode `case` with `binary`; the encoder's stderr (the seams' call counters) is appended
    to the list `log` when given."""
    cfg, kind, frames, qp = CASES[case][:4]
    extra = CASES[case][6] if len(CASES[case]) > 6 else []
    w, h = case_size(case)
    yuv = os.path.join(tmp, f"{kind}_{w}x{h}.yuv")
    if kind == "foreman":  # the reference's own clip (176x144, 3 frames)
        yuv = os.path.join(ROOT, "tests", "golden", "foreman_part_qcif.yuv")
    elif not os.path.exists(yuv):
        make_yuv.write_yuv(yuv, kind, w, h, YUV_FRAMES if (w, h) == (W, H) else frames)
    bs, rec = os.path.join(tmp, case + ".bin"), os.path.join(tmp, case + ".rec.yuv")
    # the encoder's per-picture lines go to HVX_SEAM_LOG_DIR/<case>.log when set (progress of a long run)
    log_dir = os.environ.get("HVX_SEAM_LOG_DIR")
    out = open(os.path.join(log_dir, case + ".log"), "w") if log_dir else subprocess.DEVNULL
    try:
        p = subprocess.run([binary, "-c", os.path.join(HERE, cfg), "-i", yuv, "-wdt", str(w), "-hgt", str(h), "-fr",
                            "30", "-f", str(frames), "-q", str(qp), "-b", bs, "-o", rec] + list(extra),
                           stdout=out, stderr=subprocess.PIPE, text=True)
    finally:
        if log_dir:
            out.close()
    if log is not None:
        log.append(p.stderr)
    if p.returncode:
        raise RuntimeError(f"{binary} failed ({p.returncode}): {p.stderr[-2000:]}")
    md5 = lambda p: hashlib.md5(open(p, "rb").read()).hexdigest()
    return {"bitstream_md5": md5(bs), "recon_md5": md5(rec)}


if __name__ == "__main__":
    exe = os.path.join(ROOT, "oracle", "_ref", "TAppEncoder")
    path = os.path.join(HERE, "expected_md5.json")
    res = json.load(open(path)) if os.path.exists(path) else {}
    todo = sys.argv[1:] or list(CASES)
    with tempfile.TemporaryDirectory() as tmp:
        for c in todo:
            res[c] = encode(exe, c, tmp)
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))

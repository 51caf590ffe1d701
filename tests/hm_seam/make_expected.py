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

CASES = {  # name: (cfg, yuv kind, frames, qp)
    "intra_rand_qp32": ("intra.cfg", "random", 1, 32),
    "intra_smooth_qp22": ("intra.cfg", "smooth", 1, 22),
    "ldp_smooth_qp32": ("ldp.cfg", "smooth", 3, 32),
    "ldb_smooth_qp32": ("ldb.cfg", "smooth", 3, 32),  # B slices: bi-prediction, identical-motion shortcut
    "ldp_rand_qp32": ("ldp.cfg", "random", 2, 32),    # uniform random: long TZ raster searches
    "ra_smooth_qp27": ("ra.cfg", "smooth", 9, 27),    # GOP8 hierarchical B: future refs, bBi refinement
    "ra_texture_qp32": ("ra.cfg", "texture", 9, 32),  # textured content in motion: uni-L0 / uni-L1 / bi AMVP choices
}
YUV_FRAMES = max(c[2] for c in CASES.values())
W, H = 416, 240


def encode(binary, case, tmp, log=None):
    """Encode `case` with `binary`; the encoder's stderr (the seams' call counters) is appended
    to the list `log` when given."""
    cfg, kind, frames, qp = CASES[case]
    yuv = os.path.join(tmp, f"{kind}.yuv")
    if not os.path.exists(yuv):
        make_yuv.write_yuv(yuv, kind, W, H, YUV_FRAMES)
    bs, rec = os.path.join(tmp, case + ".bin"), os.path.join(tmp, case + ".rec.yuv")
    # the encoder's per-picture lines go to HVX_SEAM_LOG_DIR/<case>.log when set (progress of a long run)
    log_dir = os.environ.get("HVX_SEAM_LOG_DIR")
    out = open(os.path.join(log_dir, case + ".log"), "w") if log_dir else subprocess.DEVNULL
    try:
        p = subprocess.run([binary, "-c", os.path.join(HERE, cfg), "-i", yuv, "-wdt", str(W), "-hgt", str(H), "-fr",
                            "30", "-f", str(frames), "-q", str(qp), "-b", bs, "-o", rec],
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
    with tempfile.TemporaryDirectory() as tmp:
        res = {c: encode(exe, c, tmp) for c in CASES}
    json.dump(res, open(os.path.join(HERE, "expected_md5.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))

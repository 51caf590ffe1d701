/* hvx_oracle_cu.c -- CPU restatement of HM-16.5rc1's CTU mode decision, TEncCu::compressCtu
 * (TEncCu.cpp:228), and of the CTU syntax walk TEncCu::encodeCtu (TEncCu.cpp:252) that carries
 * the CABAC contexts from CTU to CTU (TEncSlice.cpp:814-828).
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the HM-exact CTU path: tests/ and
 * __graft_entry__.smoke() call it as the checker; it is never the product path.  It is pinned
 * against the reference's own decisions captured by oracle/cu_capture.cpp (tests/golden/ctu_*.bin):
 * per CTU the whole TComDataCU, the coefficients, the reconstruction and the RD totals.
 *
 * Scope: 4:2:0 8-bit Main profile as the reference's encoder_lowdelay_P_main.cfg /
 * encoder_randomaccess_main.cfg / encoder_intra_main.cfg configure it: CTU 64, max depth 4,
 * TU 4..32 with QuadtreeTUMaxDepthInter/Intra 3, RDOQ + RDOQTS, sign hiding, TransformSkip +
 * TransformSkipFast, FEN, FDM, AMP (AMP_ENC_SPEEDUP + AMP_MRG), TZ search SR 64, HadamardME,
 * TMVP, 5 merge candidates, no ECU/ESD/CFM, no PCM, no delta QP, no lossless, no weighted
 * prediction, one slice and one tile, WPP off.  Uni-prediction (P slices) and the I slice path.
 *
 * Every function cites the reference function it restates (paths under hm-16.5rc1/source/Lib).
 * Leaf kernels are the pinned restatements of hvx_oracle.c (ME, MC, transformNxN / RDOQ,
 * invTransformNxN, codeCoeffNxN, estBit, intra prediction and its first pass).
 */
#include <assert.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hvx_oracle.h"
#include "hvx_oracle_cu.h"

#define MAX_DOUBLE 1.7e+308
#define MAXU32 0xffffffffu

enum { SIZE_2Nx2N, SIZE_2NxN, SIZE_Nx2N, SIZE_NxN, SIZE_2NxnU, SIZE_2NxnD, SIZE_nLx2N, SIZE_nRx2N, SIZE_NONE };
enum { MODE_INTER = 0, MODE_INTRA = 1, MODE_NONE = 2 };
enum { CI_CURR_BEST, CI_NEXT_BEST, CI_TEMP_BEST, CI_CHROMA_INTRA, CI_QT_TRAFO_TEST, CI_QT_TRAFO_ROOT, CI_NUM };
enum { B_SLICE = 0, P_SLICE = 1, I_SLICE = 2 };
#define DM_CHROMA_IDX 36

/* context buffer offsets in TEncSbac::m_contextModels (constructor order TEncSbac.cpp:62-92) */
enum {
  X_SPLIT = 0, X_SKIP = 3, X_MERGE_FLAG = 6, X_MERGE_IDX = 7, X_PART = 8, X_PRED = 12, X_INTRA = 13, X_CHROMA = 14,
  X_INTER_DIR = 19, X_REF = 24, X_MVD = 26, X_QT_CBF = 28, X_SUBDIV = 38, X_ROOT_CBF = 41, X_MVP = 180
};

/* ============================================================================================
 * Tables: z-scan / raster orders of the 16x16 4x4-partition grid of a CTU (TComRom.cpp:196-260)
 * ========================================================================================== */
static int Z2R[256], R2Z[256];
static void tables_init(void) {
  static int done = 0;
  if (done) return;
  for (int z = 0; z < 256; z++) {
    int x = 0, y = 0;
    for (int b = 0; b < 4; b++) { x |= ((z >> (2 * b)) & 1) << b; y |= ((z >> (2 * b + 1)) & 1) << b; }
    Z2R[z] = y * 16 + x;
    R2Z[y * 16 + x] = z;
  }
  done = 1;
}
#define RPX(r) (((r) & 15) << 2)
#define RPY(r) (((r) >> 4) << 2)

/* ============================================================================================
 * CABAC bit counter: TEncBinCABACCounter (TEncBinCoderCABACCounter.cpp:74-120) over the 202
 * contexts of TEncSbac; a coder is the context states plus the counter's m_fracBits, which
 * TEncSbac::load/store copy together (TEncSbac.cpp:396-425, TEncBinCoderCABAC.cpp:150).
 * ========================================================================================== */
static const uint8_t kLpsNext[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                     13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                     24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                     33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};
typedef hvxo_hm_coder coder_t;

typedef struct hm_enc hm_enc;
static void cbin(hm_enc *e, int ctx, int v);
static void cep(hm_enc *e, int n);
static void ctrm(hm_enc *e, int v);

/* ============================================================================================
 * CU data: TComDataCU's per-partition arrays (TComDataCU.h) for a CU object of any depth,
 * indexed by the partition's z-order index relative to the CU (m_absZIdxInCtu + rel).
 * ========================================================================================== */
typedef struct {
  int8_t depth, part, pred, skip, merge, merge_idx, inter_dir, tr_idx;
  int8_t ref[2], mvp_idx[2], mvp_num[2];
  int16_t mv[2][2], mvd[2][2];
  uint8_t idir[2], ts[3], cbf[3], width;
  int8_t qp;
} hm_part;

typedef struct {
  int depth, zidx, x, y, ctu, nparts, width;
  hm_part p[256];
  int32_t coef[3][4096];
  uint32_t bits, dist;
  double cost;
  double dssim;   /* HVX_RD_SSIM: the SSIM distortion of the CU's reconstruction (cu_dssim) */
  int merge_amp;
} hm_cu;

struct hvxo_hm_ctu_data {
  hm_part p[256];
  int32_t coef[3][4096];
  uint32_t bits, dist;
  double cost;
};

typedef struct { int16_t c[3][64 * 64]; } yuv_t;  /* TComYuv of a max CU: Y stride 64, Cb/Cr stride 32 */
static inline int ystride(int c) { return c ? 32 : 64; }
static inline int16_t *yaddr(yuv_t *b, int c, int x, int y) { return b->c[c] + y * ystride(c) + x; }

/* ============================================================================================
 * The encoder: TEncCu + TEncSearch + TComTrQuant state the decision of one CTU reads and writes.
 * ========================================================================================== */
struct hm_enc {
  const hvxo_hm_pic *pic;
  hvxo_hm_ctu_data *ctus;      /* the picture's CTU data (TComPic::getCtu), written by copyToPic */
  int16_t *rec[3];             /* the picture reconstruction (TComPicYuv rec), sample (0,0), stride rs[c] */
  int rs[3];
  hm_cu cu_store[2][4];
  hm_cu *best[4], *temp[4];
  yuv_t yuv_store[8][4];
  yuv_t *orig[4], *pred_best[4], *pred_temp[4], *resi_best[4], *resi_temp[4], *reco_best[4], *reco_temp[4];
  coder_t rd[6][CI_NUM];      /* m_pppcRDSbacCoder[depth][CI_*] */
  coder_t *cur;               /* the coder the entropy calls count with (m_pcRDGoOnSbacCoder or rd[..]) */
  coder_t goon;
  hvx_estbits est;            /* TComTrQuant::m_pcEstBitsSbac */
  int16_t int2n[2][4][2];     /* TEncSearch::m_integerMv2Nx2N */
  int32_t qt_coef[3][4][4096];/* m_ppcQTTempCoeff[comp][layer] */
  yuv_t qt_yuv[4];            /* m_pcQTTempTComYuv[layer] */
  int32_t qt_tu_coef[3][1024];/* m_pcQTTempTUCoeff */
  yuv_t qt_ts_yuv;            /* m_pcQTTempTransformSkipTComYuv */
  int16_t shared_pred[3][1024];
  uint8_t tmp_tridx[256], tmp_cbf[3][256], tmp_ts[3][256];
  yuv_t yuv_pred_l[2], yuv_pred_tmp, tmp_yuv_pred; /* m_acYuvPred, m_cYuvPredTemp, m_tmpYuvPred */
  int ctu_addr, ctu_x, ctu_y;
  int slice_qp;
  int slice_start, slice_end;  /* SliceMode=1 slice of the CTU (CTU addresses) */
};

static void cbin(hm_enc *e, int ctx, int v) {
  coder_t *c = e->cur;
  const int s = c->st[ctx], p = s >> 1, mps = s & 1;
  c->frac += (uint64_t)e->pic->entropy_bits[s ^ v];
  if (v == mps) c->st[ctx] = (uint8_t)(((p < 62 ? p + 1 : p) << 1) | mps);
  else c->st[ctx] = (uint8_t)((kLpsNext[p] << 1) | (p == 0 ? mps ^ 1 : mps));
}
static void cep(hm_enc *e, int n) { e->cur->frac += 32768ull * (uint64_t)n; }
static void ctrm(hm_enc *e, int v) { e->cur->frac += (uint64_t)e->pic->entropy_bits[126 ^ v]; } /* getEntropyBitsTrm */
static void reset_bits(hm_enc *e) { e->cur->frac &= 32767; }                      /* TEncBinCABAC::resetBits */
static uint32_t written_bits(hm_enc *e) { return (uint32_t)(e->cur->frac >> 15); } /* getNumWrittenBits */
static void load(coder_t *dst, const coder_t *src) { *dst = *src; }

/* ============================================================================================
 * Neighbour access: TComDataCU::getPULeft / getPUAbove / getPUAboveLeft / getPUBelowLeft /
 * getPUAboveRight (TComDataCU.cpp:1024-1238).  A result is the CU object holding the partition
 * (the current CU for partitions inside it, else the picture's CTU) and the partition index in
 * that object.
 * ========================================================================================== */
typedef struct { const hm_part *p; int idx; int valid; } nb_t;

static const hm_part *ctu_parts(const hm_enc *e, int addr) { return e->ctus[addr].p; }
/* getCtuLeft / ... with CUIsFromSameSliceAndTile: a CTU before the slice is unavailable */
static int in_slice(const hm_enc *e, int a) { return a >= e->slice_start ? a : -1; }
static int ctu_left(const hm_enc *e) { return e->ctu_x > 0 ? in_slice(e, e->ctu_addr - 1) : -1; }
static int ctu_above(const hm_enc *e) { return e->ctu_y > 0 ? in_slice(e, e->ctu_addr - e->pic->w_ctus) : -1; }
static int ctu_above_left(const hm_enc *e) {
  return (e->ctu_x > 0 && e->ctu_y > 0) ? in_slice(e, e->ctu_addr - e->pic->w_ctus - 1) : -1;
}
static int ctu_above_right(const hm_enc *e) {
  return (e->ctu_y > 0 && e->ctu_x < e->pic->w_ctus - 1) ? in_slice(e, e->ctu_addr - e->pic->w_ctus + 1) : -1;
}
static nb_t nb_none(void) { nb_t n = {NULL, 0, 0}; return n; }
static nb_t nb_make(const hm_part *p, int idx) { nb_t n = {p, idx, 1}; return n; }

static nb_t get_pu_left(const hm_enc *e, const hm_cu *cu, int cur) {
  const int r = Z2R[cur], rc = Z2R[cu->zidx];
  if ((r & 15) != 0) {
    const int z = R2Z[r - 1];
    if ((r & 15) == (rc & 15)) return nb_make(ctu_parts(e, e->ctu_addr), z);
    return nb_make(cu->p, z - cu->zidx);
  }
  const int a = ctu_left(e);
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(e, a), R2Z[r + 15]);
}
static nb_t get_pu_above(const hm_enc *e, const hm_cu *cu, int cur, int planar_at_ctu_boundary) {
  const int r = Z2R[cur], rc = Z2R[cu->zidx];
  if ((r >> 4) != 0) {
    const int z = R2Z[r - 16];
    if ((r >> 4) == (rc >> 4)) return nb_make(ctu_parts(e, e->ctu_addr), z);
    return nb_make(cu->p, z - cu->zidx);
  }
  if (planar_at_ctu_boundary) return nb_none();
  const int a = ctu_above(e);
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(e, a), R2Z[r + 256 - 16]);
}
static nb_t get_pu_above_left(const hm_enc *e, const hm_cu *cu, int cur) {
  const int r = Z2R[cur], rc = Z2R[cu->zidx];
  if ((r & 15) != 0) {
    if ((r >> 4) != 0) {
      const int z = R2Z[r - 17];
      if ((r & 15) == (rc & 15) || (r >> 4) == (rc >> 4)) return nb_make(ctu_parts(e, e->ctu_addr), z);
      return nb_make(cu->p, z - cu->zidx);
    }
    const int a = ctu_above(e);
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(e, a), R2Z[r + 256 - 16 - 1]);
  }
  if ((r >> 4) != 0) {
    const int a = ctu_left(e);
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(e, a), R2Z[r - 1]);
  }
  const int a = ctu_above_left(e);
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(e, a), R2Z[255]);
}
/* :1141 -- cur is the PU's bottom-left partition; offset in units */
static nb_t get_pu_below_left(const hm_enc *e, const hm_cu *cu, int cur, int off) {
  const int r = Z2R[cur];
  const int rc_lb = Z2R[cu->zidx] + ((cu->width >> 2) - 1) * 16;
  if (e->ctu_y * 64 + RPY(r) + 4 * off >= e->pic->h) return nb_none();
  if ((r >> 4) < 16 - off) {
    if ((r & 15) != 0) {
      const int zz = R2Z[r + off * 16 - 1];
      if (cur > zz) {
        if ((r & 15) == (rc_lb & 15) || (r >> 4) == (rc_lb >> 4)) return nb_make(ctu_parts(e, e->ctu_addr), zz);
        return nb_make(cu->p, zz - cu->zidx);
      }
      return nb_none();
    }
    const int a = ctu_left(e);
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(e, a), R2Z[r + (1 + off) * 16 - 1]);
  }
  return nb_none();
}
/* :1185 -- cur is the PU's top-right partition */
static nb_t get_pu_above_right(const hm_enc *e, const hm_cu *cu, int cur, int off) {
  const int r = Z2R[cur];
  const int rc_rt = Z2R[cu->zidx] + (cu->width >> 2) - 1;
  if (e->ctu_x * 64 + RPX(r) + 4 * off >= e->pic->w) return nb_none();
  if ((r & 15) < 16 - off) {
    if ((r >> 4) != 0) {
      const int zz = R2Z[r - 16 + off];
      if (cur > zz) {
        if ((r & 15) == (rc_rt & 15) || (r >> 4) == (rc_rt >> 4)) return nb_make(ctu_parts(e, e->ctu_addr), zz);
        return nb_make(cu->p, zz - cu->zidx);
      }
      return nb_none();
    }
    const int a = ctu_above(e);
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(e, a), R2Z[r + 256 - 16 + off]);
  }
  if ((r >> 4) != 0) return nb_none();
  const int a = ctu_above_right(e);
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(e, a), R2Z[256 - 16 + off - 1]);
}
static inline int nb_inter(nb_t n) { return n.valid && n.p[n.idx].pred == MODE_INTER; }
static inline int nb_intra(nb_t n) { return n.valid && n.p[n.idx].pred == MODE_INTRA; }

/* ============================================================================================
 * Partition geometry: getPartIndexAndSize (:1893), getPartPosition (:2555),
 * deriveLeftRightTopIdx(General) / deriveLeftBottomIdx(General) / deriveRightBottomIdx
 * (:1947-2157), xDeriveCenterIdx (:3152).  Indices are CTU-absolute z-order.
 * ========================================================================================== */
static int num_parts_of(int ps) { return ps == SIZE_2Nx2N ? 1 : ps == SIZE_NxN ? 4 : 2; }
static void part_index_size(const hm_cu *cu, int ps, int pu, int *addr, int *w, int *h) {
  const int W = cu->width, N = cu->nparts;
  switch (ps) {
    case SIZE_2NxN: *w = W; *h = W >> 1; *addr = pu ? N >> 1 : 0; break;
    case SIZE_Nx2N: *w = W >> 1; *h = W; *addr = pu ? N >> 2 : 0; break;
    case SIZE_NxN: *w = W >> 1; *h = W >> 1; *addr = (N >> 2) * pu; break;
    case SIZE_2NxnU: *w = W; *h = pu ? (W >> 2) + (W >> 1) : W >> 2; *addr = pu ? N >> 3 : 0; break;
    case SIZE_2NxnD: *w = W; *h = pu ? W >> 2 : (W >> 2) + (W >> 1); *addr = pu ? (N >> 1) + (N >> 3) : 0; break;
    case SIZE_nLx2N: *w = pu ? (W >> 2) + (W >> 1) : W >> 2; *h = W; *addr = pu ? N >> 4 : 0; break;
    case SIZE_nRx2N: *w = pu ? W >> 2 : (W >> 2) + (W >> 1); *h = W; *addr = pu ? (N >> 2) + (N >> 4) : 0; break;
    default: *w = W; *h = W; *addr = 0; break;
  }
}
static void part_position(const hm_cu *cu, int ps, int pu, int *xp, int *yp, int *w, int *h) {
  const int W = cu->width;
  int a;
  part_index_size(cu, ps, pu, &a, w, h);
  *xp = cu->x;
  *yp = cu->y;
  switch (ps) {
    case SIZE_2NxN: case SIZE_2NxnU: case SIZE_2NxnD: *yp = pu ? cu->y + W - *h : cu->y; break;
    case SIZE_Nx2N: case SIZE_nLx2N: case SIZE_nRx2N: *xp = pu ? cu->x + W - *w : cu->x; break;
    case SIZE_NxN: *xp = cu->x + (pu & 1) * *w; *yp = cu->y + (pu >> 1) * *h; break;
    default: break;
  }
}
/* the LT / RT / LB partitions of a PU from its geometry (equal to the reference's derivations) */
static void pu_corners(const hm_cu *cu, int ps, int pu, int *lt, int *rt, int *lb) {
  int a, w, h;
  part_index_size(cu, ps, pu, &a, &w, &h);
  const int r = Z2R[cu->zidx + a];
  *lt = cu->zidx + a;
  *rt = R2Z[r + (w >> 2) - 1];
  *lb = R2Z[r + ((h >> 2) - 1) * 16];
}
/* deriveRightBottomIdx (:2123): the partition at the PU's bottom-right sample */
static int pu_right_bottom(const hm_cu *cu, int ps, int pu) {
  int a, w, h;
  part_index_size(cu, ps, pu, &a, &w, &h);
  const int r = Z2R[cu->zidx + a];
  return R2Z[r + ((h >> 2) - 1) * 16 + (w >> 2) - 1];
}
static int pu_center(const hm_cu *cu, int ps, int pu) {
  int a, w, h;
  part_index_size(cu, ps, pu, &a, &w, &h);
  return R2Z[Z2R[cu->zidx + a] + ((h >> 2) / 2) * 16 + (w >> 2) / 2];
}

/* ============================================================================================
 * Sub-part setters: TComDataCU::setSubPart over a PU (:1701) and the *SubParts family
 * ========================================================================================== */
static void pu_range_apply(hm_cu *cu, int ps, int pu, void (*fn)(hm_part *, const void *), const void *arg) {
  int a, w, h;
  part_index_size(cu, ps, pu, &a, &w, &h);
  const int r0 = Z2R[cu->zidx + a];
  for (int y = 0; y < (h >> 2); y++)
    for (int x = 0; x < (w >> 2); x++) fn(&cu->p[R2Z[r0 + y * 16 + x] - cu->zidx], arg);
}
typedef struct { int list; int16_t mv[2]; int ref; } mvf_arg;
static void set_mvfield_fn(hm_part *p, const void *a) {
  const mvf_arg *m = (const mvf_arg *)a;
  p->mv[m->list][0] = m->mv[0]; p->mv[m->list][1] = m->mv[1]; p->ref[m->list] = (int8_t)m->ref;
}
static void set_mv_fn(hm_part *p, const void *a) {
  const mvf_arg *m = (const mvf_arg *)a;
  p->mv[m->list][0] = m->mv[0]; p->mv[m->list][1] = m->mv[1];
}
static void set_ref_fn(hm_part *p, const void *a) { const mvf_arg *m = (const mvf_arg *)a; p->ref[m->list] = (int8_t)m->ref; }
static void set_mvd_fn(hm_part *p, const void *a) {
  const mvf_arg *m = (const mvf_arg *)a;
  p->mvd[m->list][0] = m->mv[0]; p->mvd[m->list][1] = m->mv[1];
}
static void pu_set_mvfield(hm_cu *cu, int ps, int pu, int list, int mx, int my, int ref) {
  mvf_arg m = {list, {(int16_t)mx, (int16_t)my}, ref};
  pu_range_apply(cu, ps, pu, set_mvfield_fn, &m);
}
static void pu_set_mv(hm_cu *cu, int ps, int pu, int list, int mx, int my) {
  mvf_arg m = {list, {(int16_t)mx, (int16_t)my}, 0};
  pu_range_apply(cu, ps, pu, set_mv_fn, &m);
}
static void pu_set_ref(hm_cu *cu, int ps, int pu, int list, int ref) {
  mvf_arg m = {list, {0, 0}, ref};
  pu_range_apply(cu, ps, pu, set_ref_fn, &m);
}
static void pu_set_mvd(hm_cu *cu, int ps, int pu, int list, int mx, int my) {
  mvf_arg m = {list, {(int16_t)mx, (int16_t)my}, 0};
  pu_range_apply(cu, ps, pu, set_mvd_fn, &m);
}
typedef struct { int which, v, list; } byte_arg;
static void set_byte_fn(hm_part *p, const void *a) {
  const byte_arg *b = (const byte_arg *)a;
  switch (b->which) {
    case 0: p->merge = (int8_t)b->v; break;
    case 1: p->merge_idx = (int8_t)b->v; break;
    case 2: p->inter_dir = (int8_t)b->v; break;
    case 3: p->mvp_idx[b->list] = (int8_t)b->v; break;
    case 4: p->mvp_num[b->list] = (int8_t)b->v; break;
  }
}
static void pu_set(hm_cu *cu, int ps, int pu, int which, int list, int v) {
  byte_arg b = {which, v, list};
  pu_range_apply(cu, ps, pu, set_byte_fn, &b);
}
#define PU_MERGE 0
#define PU_MERGE_IDX 1
#define PU_INTER_DIR 2
#define PU_MVP_IDX 3
#define PU_MVP_NUM 4

static void cu_set_all(hm_cu *cu, int field, int v) {
  for (int i = 0; i < cu->nparts; i++) {
    hm_part *p = &cu->p[i];
    switch (field) {
      case 0: p->part = (int8_t)v; break;
      case 1: p->pred = (int8_t)v; break;
      case 2: p->skip = (int8_t)v; break;
      case 3: p->tr_idx = (int8_t)v; break;
    }
  }
}
#define F_PART 0
#define F_PRED 1
#define F_SKIP 2
#define F_TRIDX 3

/* initEstData (:552) */
static void cu_init_est(hm_cu *cu, int qp) {
  for (int i = 0; i < cu->nparts; i++) {
    hm_part *p = &cu->p[i];
    memset(p, 0, sizeof(*p));
    p->mvp_idx[0] = p->mvp_idx[1] = -1;
    p->mvp_num[0] = p->mvp_num[1] = -1;
    p->depth = (int8_t)cu->depth;
    p->width = (uint8_t)cu->width;
    p->part = SIZE_NONE;
    p->pred = MODE_NONE;
    p->qp = (int8_t)qp;
    p->idir[0] = 1; /* DC_IDX */
    p->idir[1] = 0;
    p->ref[0] = p->ref[1] = -1;
  }
  const int n = cu->width * cu->width;
  memset(cu->coef[0], 0, sizeof(int32_t) * n);
  memset(cu->coef[1], 0, sizeof(int32_t) * (n >> 2));
  memset(cu->coef[2], 0, sizeof(int32_t) * (n >> 2));
  cu->bits = 0; cu->dist = 0; cu->cost = MAX_DOUBLE; cu->dssim = 0;
}
/* initSubCU (:623) / initCtu (:434): geometry, then the same resets */
static void cu_init_sub(hm_cu *cu, const hm_cu *parent, int idx, int depth, int qp) {
  cu->depth = depth;
  cu->width = 64 >> depth;
  cu->nparts = 256 >> (2 * depth);
  cu->zidx = parent->zidx + (parent->nparts >> 2) * idx;
  cu->x = parent->x + cu->width * (idx & 1);
  cu->y = parent->y + cu->width * (idx >> 1);
  cu->ctu = parent->ctu;
  cu_init_est(cu, qp);
}
/* copyPartFrom (:859) */
static void cu_copy_part_from(hm_cu *dst, const hm_cu *src, int idx, int depth) {
  dst->cost += src->cost;
  dst->dist += src->dist;
  dst->dssim += src->dssim;
  dst->bits += src->bits;
  const int off = src->nparts * idx;
  memcpy(&dst->p[off], src->p, sizeof(hm_part) * src->nparts);
  const int ny = (64 * 64) >> (depth << 1);
  memcpy(dst->coef[0] + idx * ny, src->coef[0], sizeof(int32_t) * ny);
  memcpy(dst->coef[1] + idx * (ny >> 2), src->coef[1], sizeof(int32_t) * (ny >> 2));
  memcpy(dst->coef[2] + idx * (ny >> 2), src->coef[2], sizeof(int32_t) * (ny >> 2));
}
/* copyToPic (:945) */
static void cu_copy_to_pic(hm_enc *e, const hm_cu *cu) {
  hvxo_hm_ctu_data *d = &e->ctus[e->ctu_addr];
  d->cost = cu->cost; d->dist = cu->dist; d->bits = cu->bits;
  memcpy(&d->p[cu->zidx], cu->p, sizeof(hm_part) * cu->nparts);
  const int ny = (64 * 64) >> (cu->depth << 1), off = cu->zidx * 16;
  memcpy(d->coef[0] + off, cu->coef[0], sizeof(int32_t) * ny);
  memcpy(d->coef[1] + (off >> 2), cu->coef[1], sizeof(int32_t) * (ny >> 2));
  memcpy(d->coef[2] + (off >> 2), cu->coef[2], sizeof(int32_t) * (ny >> 2));
}
static int cu_qt_root_cbf(const hm_cu *cu, int i) { return cu->p[i].cbf[0] & 1 || cu->p[i].cbf[1] & 1 || cu->p[i].cbf[2] & 1; }
static inline int cbf_at(const hm_part *p, int comp, int depth) { return (p->cbf[comp] >> depth) & 1; }

/* ============================================================================================
 * Syntax elements counted by TEncBinCABACCounter: TEncSbac.cpp:427-1104
 * ========================================================================================== */
/* getCtxSplitFlag (TComDataCU.cpp:1487) */
static int ctx_split_flag(const hm_enc *e, const hm_cu *cu, int rel, int depth) {
  nb_t l = get_pu_left(e, cu, cu->zidx + rel), a = get_pu_above(e, cu, cu->zidx + rel, 0);
  return (l.valid && l.p[l.idx].depth > depth) + (a.valid && a.p[a.idx].depth > depth);
}
/* codeSplitFlag (:613) */
static void code_split_flag(hm_enc *e, const hm_cu *cu, int rel, int depth) {
  if (depth == 3) return;
  cbin(e, X_SPLIT + ctx_split_flag(e, cu, rel, depth), cu->p[rel].depth > depth);
}
/* codeSkipFlag (:543) with getCtxSkipFlag (TComDataCU.cpp:1545) */
static void code_skip_flag(hm_enc *e, const hm_cu *cu, int rel) {
  if (e->pic->slice_type == I_SLICE) return;
  nb_t l = get_pu_left(e, cu, cu->zidx + rel), a = get_pu_above(e, cu, cu->zidx + rel, 0);
  const int ctx = (l.valid && l.p[l.idx].skip) + (a.valid && a.p[a.idx].skip);
  cbin(e, X_SKIP + ctx, cu->p[rel].skip ? 1 : 0);
}
static void code_merge_flag(hm_enc *e, const hm_cu *cu, int rel) { cbin(e, X_MERGE_FLAG, cu->p[rel].merge ? 1 : 0); }
/* codeMergeIndex (:583) */
static void code_merge_index(hm_enc *e, const hm_cu *cu, int rel) {
  const int idx = cu->p[rel].merge_idx, n = e->pic->max_merge;
  if (n > 1)
    for (int i = 0; i < n - 1; i++) {
      const int sym = i == idx ? 0 : 1;
      if (i == 0) cbin(e, X_MERGE_IDX, sym);
      else cep(e, 1);
      if (!sym) break;
    }
}
static void code_pred_mode(hm_enc *e, const hm_cu *cu, int rel) {
  if (e->pic->slice_type == I_SLICE) return;
  cbin(e, X_PRED, cu->p[rel].pred == MODE_INTRA);
}
/* codePartSize (:435); AMP on, log2DiffMaxMinCodingBlockSize 3 */
static void code_part_size(hm_enc *e, const hm_cu *cu, int rel, int depth) {
  const int ps = cu->p[rel].part;
  if (cu->p[rel].pred == MODE_INTRA) {
    if (depth == 3) cbin(e, X_PART + 0, ps == SIZE_2Nx2N);
    return;
  }
  const int amp = e->pic->amp && depth < 3;
  switch (ps) {
    case SIZE_2Nx2N: cbin(e, X_PART + 0, 1); break;
    case SIZE_2NxN: case SIZE_2NxnU: case SIZE_2NxnD:
      cbin(e, X_PART + 0, 0);
      cbin(e, X_PART + 1, 1);
      if (amp) {
        if (ps == SIZE_2NxN) cbin(e, X_PART + 3, 1);
        else { cbin(e, X_PART + 3, 0); cep(e, 1); }
      }
      break;
    case SIZE_Nx2N: case SIZE_nLx2N: case SIZE_nRx2N:
      cbin(e, X_PART + 0, 0);
      cbin(e, X_PART + 1, 0);
      if (depth == 3 && cu->p[rel].width != 8) cbin(e, X_PART + 2, 1);
      if (amp) {
        if (ps == SIZE_Nx2N) cbin(e, X_PART + 3, 1);
        else { cbin(e, X_PART + 3, 0); cep(e, 1); }
      }
      break;
    case SIZE_NxN:
      if (depth == 3 && cu->p[rel].width != 8) { cbin(e, X_PART + 0, 0); cbin(e, X_PART + 1, 0); cbin(e, X_PART + 2, 0); }
      break;
  }
}
/* getIntraDirPredictor (TComDataCU.cpp:1401), luma */
static int intra_dir_predictor(const hm_enc *e, const hm_cu *cu, int rel, int *pred) {
  nb_t l = get_pu_left(e, cu, cu->zidx + rel), a = get_pu_above(e, cu, cu->zidx + rel, 1);
  const int ld = (l.valid && l.p[l.idx].pred == MODE_INTRA) ? l.p[l.idx].idir[0] : 1;
  const int ad = (a.valid && a.p[a.idx].pred == MODE_INTRA) ? a.p[a.idx].idir[0] : 1;
  if (ld == ad) {
    if (ld > 1) { pred[0] = ld; pred[1] = ((ld + 29) % 32) + 2; pred[2] = ((ld - 1) % 32) + 2; }
    else { pred[0] = 0; pred[1] = 1; pred[2] = 26; }
    return 1;
  }
  pred[0] = ld; pred[1] = ad;
  pred[2] = (ld && ad) ? 0 : ((ld + ad) < 2 ? 26 : 1);
  return 2;
}
/* codeIntraDirLumaAng (:643) */
static void code_intra_dir_luma(hm_enc *e, const hm_cu *cu, int rel, int multiple) {
  const int npu = (multiple && cu->p[rel].part == SIZE_NxN) ? 4 : 1;
  const int off = (256 >> (2 * cu->p[rel].depth)) >> 2;
  int dir[4], preds[4][3], pidx[4];
  for (int j = 0; j < npu; j++) {
    dir[j] = cu->p[rel + off * j].idir[0];
    intra_dir_predictor(e, cu, rel + off * j, preds[j]);
    pidx[j] = -1;
    for (int i = 0; i < 3; i++)
      if (dir[j] == preds[j][i]) pidx[j] = i;
    cbin(e, X_INTRA, pidx[j] != -1);
  }
  for (int j = 0; j < npu; j++) {
    if (pidx[j] != -1) cep(e, pidx[j] ? 2 : 1);
    else cep(e, 5);
  }
}
/* codeIntraDirChroma (:698) */
static void code_intra_dir_chroma(hm_enc *e, const hm_cu *cu, int rel) {
  if (cu->p[rel].idir[1] == DM_CHROMA_IDX) cbin(e, X_CHROMA, 0);
  else { cbin(e, X_CHROMA, 1); cep(e, 2); }
}
/* codeRefFrmIdx (:748) */
static void code_ref_idx(hm_enc *e, const hm_cu *cu, int rel, int list) {
  int r = cu->p[rel].ref[list];
  cbin(e, X_REF + 0, r == 0 ? 0 : 1);
  if (r > 0) {
    const int n = e->pic->nref[list] - 2;
    r--;
    for (int i = 0; i < n; i++) {
      const int sym = i == r ? 0 : 1;
      if (i == 0) cbin(e, X_REF + 1, sym);
      else cep(e, 1);
      if (!sym) break;
    }
  }
}
/* xWriteEpExGolomb (:308) bin count */
static int ep_exgolomb_bins(uint32_t sym, int k) {
  int n = 0;
  while (sym >= (1u << k)) { n++; sym -= 1u << k; k++; }
  return n + 1 + k;
}
/* codeMvd (:779) */
static void code_mvd(hm_enc *e, const hm_cu *cu, int rel, int list) {
  if (e->pic->mvd_l1_zero && list == 1 && cu->p[rel].inter_dir == 3) return;
  const int h = cu->p[rel].mvd[list][0], v = cu->p[rel].mvd[list][1];
  cbin(e, X_MVD + 0, h != 0);
  cbin(e, X_MVD + 0, v != 0);
  const int ah = abs(h), av = abs(v);
  if (h) cbin(e, X_MVD + 1, ah > 1);
  if (v) cbin(e, X_MVD + 1, av > 1);
  if (h) { if (ah > 1) cep(e, ep_exgolomb_bins((uint32_t)(ah - 2), 1)); cep(e, 1); }
  if (v) { if (av > 1) cep(e, ep_exgolomb_bins((uint32_t)(av - 2), 1)); cep(e, 1); }
}
/* codeMVPIdx (:427): xWriteUnaryMaxSymbol(idx, ctx, 1, 1) */
static void code_mvp_idx(hm_enc *e, const hm_cu *cu, int rel, int list) { cbin(e, X_MVP, cu->p[rel].mvp_idx[list] ? 1 : 0); }
/* codeInterDir (:729) */
static void code_inter_dir(hm_enc *e, const hm_cu *cu, int rel) {
  const int d = cu->p[rel].inter_dir - 1, ctx = cu->p[rel].depth;
  if (cu->p[rel].part == SIZE_2Nx2N || cu->p[rel].width != 8) { /* getHeight(abs): the CU height at the partition */
    cbin(e, X_INTER_DIR + ctx, d == 2);
  }
  if (d < 2) cbin(e, X_INTER_DIR + 4, d);
}
/* encodePUWise (TEncEntropy.cpp:457) */
static void encode_pu_wise(hm_enc *e, const hm_cu *cu, int rel) {
  const int ps = cu->p[rel].part, npu = num_parts_of(ps);
  static const int pu_off16[8] = {0, 8, 4, 4, 2, 10, 1, 5}; /* g_auiPUOffset */
  const int puoff = (pu_off16[ps] << ((4 - cu->p[rel].depth) << 1)) >> 4;
  for (int pu = 0, sub = rel; pu < npu; pu++, sub += puoff) {
    code_merge_flag(e, cu, sub);
    if (cu->p[sub].merge) code_merge_index(e, cu, sub);
    else {
      if (e->pic->slice_type == B_SLICE) code_inter_dir(e, cu, sub);
      for (int l = 0; l < 2; l++)
        if (e->pic->nref[l] > 0) {
          if (e->pic->nref[l] != 1 && (cu->p[sub].inter_dir & (1 << l))) code_ref_idx(e, cu, sub, l);
          if (cu->p[sub].inter_dir & (1 << l)) code_mvd(e, cu, sub, l);
          if (cu->p[sub].inter_dir & (1 << l)) code_mvp_idx(e, cu, sub, l);
        }
    }
  }
}
/* encodePredInfo (TEncEntropy.cpp:427) */
static void encode_pred_info(hm_enc *e, const hm_cu *cu, int rel) {
  if (cu->p[rel].pred == MODE_INTRA) {
    code_intra_dir_luma(e, cu, rel, 1);
    code_intra_dir_chroma(e, cu, rel);
  } else encode_pu_wise(e, cu, rel);
}

/* ============================================================================================
 * Transform-unit recursion: TComTU / TComTURecurse (TComTU.cpp:40-210), 4:2:0.
 * Rectangles and coefficient offsets are relative to the CU.
 * ========================================================================================== */
typedef struct tu_s {
  int cu_depth, cu_zidx;
  int split, section, last_of_level;
  int rel, step;
  int log2;
  int trd[3];
  int x0[3], y0[3], w[3], h[3], ow[3];
  int all[3];
  int off[3];
} tu_t;
static void tu_root(tu_t *t, const hm_cu *cu, int init_tr_depth) {
  memset(t, 0, sizeof(*t));
  t->cu_depth = cu->depth;
  t->cu_zidx = cu->zidx;
  t->last_of_level = 1;
  t->step = 256 >> (2 * cu->depth);
  int l = 0;
  while ((4 << l) < (64 >> (cu->depth + init_tr_depth))) l++;
  t->log2 = l + 2;
  for (int c = 0; c < 3; c++) {
    t->trd[c] = init_tr_depth;
    t->w[c] = t->h[c] = t->ow[c] = c ? cu->width >> 1 : cu->width;
    t->all[c] = 1;
  }
}
/* quad split child (the constructor with QUAD_SPLIT, :97-160) */
static void tu_child(tu_t *t, const tu_t *p, int last_of_level) {
  *t = *p;
  t->split = 2;
  t->section = 0;
  t->last_of_level = last_of_level;
  t->rel = p->all[0] ? p->rel : (p->rel & ~3);
  t->step = (p->step >> 2) > 1 ? p->step >> 2 : 1;
  t->log2 = p->log2 - 1;
  for (int c = 0; c < 3; c++) {
    t->trd[c] = p->trd[c] + 1;
    t->w[c] = p->w[c] >> 1;
    t->h[c] = p->h[c] >> 1;
    t->x0[c] = p->x0[c];
    t->y0[c] = p->y0[c];
    t->off[c] = p->off[c];
    if ((t->w[c] < 4 || t->h[c] < 4) && t->w[c] != 0) {
      t->w[c] = p->w[c];
      t->h[c] = p->h[c];
      t->all[c] = 0;
      t->trd[c]--;
    } else t->all[c] = 1;
    t->ow[c] = t->w[c];
    if (!t->all[c] && last_of_level) t->w[c] = 0;
  }
}
/* nextSection (:166) -- returns 0 after the last */
static int tu_next(tu_t *t, const tu_t *p) {
  for (int c = 0; c < 3; c++) {
    t->off[c] += t->w[c] * t->h[c];
    if (t->last_of_level) t->w[c] = t->ow[c];
    t->x0[c] += t->w[c];
    if (t->x0[c] >= p->x0[c] + p->w[c]) { t->x0[c] = p->x0[c]; t->y0[c] += t->h[c]; }
    if (!t->all[c] && (!t->last_of_level || t->section != 2)) t->w[c] = 0;
  }
  t->rel += t->step;
  t->section++;
  return t->section < 4;
}
static inline int tu_abs_rel(const tu_t *t) { return t->rel; }                       /* GetAbsPartIdxTU() - CU zidx */
static inline int tu_abs_rel_c(const tu_t *t, int c) { return t->all[c] ? t->rel : (t->rel & ~3); }
static inline int tu_nparts(const tu_t *t, int c) { return t->all[c] ? t->step : t->step * 4; }
static inline int tu_proc(const tu_t *t, int c) { return t->w[c] != 0; }
static inline int tu_depth_rel(const tu_t *t) { return t->trd[0]; }
static inline int tu_depth_total(const tu_t *t) { return t->cu_depth + t->trd[0]; }

/* getQuadtreeTULog2MinSizeInCU (TComDataCU.cpp:1518) */
static int qt_min_log2(const hm_cu *cu, int rel) {
  int l2 = 0;
  while ((1 << l2) < cu->width) l2++;
  const int intra = cu->p[rel].pred == MODE_INTRA;
  const int maxd = 3;
  const int isplit = intra && cu->p[rel].part == SIZE_NxN ? 1 : 0;
  if (l2 < 2 + maxd - 1 + isplit) return 2;
  int m = l2 - (maxd - 1 + isplit);
  return m > 5 ? 5 : m;
}
/* codeQtCbf (:920), 4:2:0 (square TUs) */
static void code_qt_cbf(hm_enc *e, const hm_cu *cu, const tu_t *t, int comp, int lowest) {
  const int ch = comp ? 1 : 0;
  const int depth = tu_depth_rel(t);
  const int ctx = ch ? depth : (depth == 0 ? 1 : 0);
  const int w = t->w[comp], h = t->h[comp];
  const int can_split = w >= 8 && h >= 8;
  const int lowest_depth = depth + ((!lowest && !can_split) ? 1 : 0);
  const int rel = tu_abs_rel_c(t, comp);
  cbin(e, X_QT_CBF + ch * 5 + ctx, cbf_at(&cu->p[rel], comp, lowest_depth));
}
static void code_qt_cbf_zero(hm_enc *e, const tu_t *t, int ch) {
  const int depth = tu_depth_rel(t);
  cbin(e, X_QT_CBF + ch * 5 + (ch ? depth : (depth == 0 ? 1 : 0)), 0);
}
static void code_subdiv(hm_enc *e, int v, int ctx) { cbin(e, X_SUBDIV + ctx, v); }

/* ============================================================================================
 * Transform units: the hvx_tu_desc of a TU (TComTrQuant state at transformNxN time) and
 * codeCoeffNxN (TEncSbac.cpp:1181) on the current coder.
 * ========================================================================================== */
static int log2i(int n) { int l = 0; while ((1 << l) < n) l++; return l; }

/* getCoefScanIdx (TComDataCU.cpp:3177), 4:2:0 */
static int coef_scan_idx(const hm_cu *cu, int rel, int w, int comp) {
  if (cu->p[rel].pred != MODE_INTRA) return 0;
  const int maxw = comp ? 4 : 8;
  if (w > maxw) return 0;
  int dir = cu->p[rel].idir[comp ? 1 : 0];
  if (dir == DM_CHROMA_IDX) dir = cu->p[comp ? (rel & ~3) : rel].idir[0];
  if (abs(dir - 26) <= 4) return 1;  /* vertical modes -> horizontal scan */
  if (abs(dir - 10) <= 4) return 2;
  return 0;
}
static void tu_desc(const hm_enc *e, const hm_cu *cu, const tu_t *t, int comp, hvx_tu_desc *d) {
  const hvxo_hm_pic *P = e->pic;
  const int rel = tu_abs_rel_c(t, comp);
  memset(d, 0, sizeof(*d));
  d->comp = comp;
  d->width = t->w[comp];
  d->height = t->h[comp];
  d->log2_size = log2i(t->h[comp]);
  d->scan_type = coef_scan_idx(cu, rel, t->w[comp], comp);
  d->use_dst = comp == 0 && cu->p[rel].pred == MODE_INTRA && t->w[0] == 4;
  d->transform_skip = cu->p[rel].ts[comp];
  d->is_intra = cu->p[rel].pred == MODE_INTRA;
  d->tr_idx = cu->p[rel].tr_idx;
  d->ctx_qt_cbf = comp ? tu_depth_rel(t) : (tu_depth_rel(t) == 0 ? 1 : 0);
  d->slice_type = P->slice_type;
  const int qp = comp ? P->chroma_qp[comp - 1] : e->slice_qp;
  d->qp_per = qp / 6;
  d->qp_rem = qp % 6;
  d->sign_hiding = 1;
  d->use_rdoq = d->use_rdoq_ts = 1;
  d->pps_tskip = 1;
  d->max_log2_tr_range = 15;
  d->bit_depth = 8;
  d->golomb_rice_stat = 0;
  d->lambda = P->tq_lambda[comp];
}
#ifdef HVXO_MEMO_STATS
/* measurement aid (not in the normal build): how often codeCoeffNxN repeats a count it made
 * recently -- same TU content, same descriptor, same context states before (FIFOs of K entries) */
#include <stdio.h>
#define MEMO_KS 6
static const int memo_k[MEMO_KS] = {1, 2, 4, 8, 16, 64};
typedef struct { int valid, w, comp, scan, ts; int32_t coef[1024]; uint8_t st[202]; } memo_e;
static memo_e memo[MEMO_KS][64];
static int memo_pos[MEMO_KS];
static long long memo_calls[6], memo_hits[MEMO_KS][6];
static void memo_report(void) {
  for (int z = 0; z < 4; z++) {
    fprintf(stderr, "memo TU %2d: %lld calls;", 4 << z, memo_calls[z]);
    for (int k = 0; k < MEMO_KS; k++) fprintf(stderr, " K=%d %.1f%%", memo_k[k], memo_calls[z] ? 100.0 * memo_hits[k][z] / memo_calls[z] : 0.0);
    fprintf(stderr, "\n");
  }
}
/* the context rows codeCoeffNxN of a channel reads or writes (TEncSbac.cpp:62-92 offsets) */
static int memo_same_ctx(const uint8_t *a, const uint8_t *b, int ch) {
  static const int lo[7][2] = {{42, 2}, {46, 27}, {90, 15}, {120, 15}, {150, 16}, {174, 4}, {183, 1}};
  static const int lc[7][2] = {{44, 2}, {74, 16}, {105, 15}, {135, 15}, {166, 8}, {178, 2}, {184, 1}};
  for (int r = 0; r < 7; r++) {
    const int o = ch ? lc[r][0] : lo[r][0], k = ch ? lc[r][1] : lo[r][1];
    if (memcmp(a + o, b + o, k)) return 0;
  }
  return 1;
}
static void memo_probe(const hvx_tu_desc *d, const int32_t *coef, const uint8_t *st) {
  static int reg = 0;
  if (!reg) { reg = 1; atexit(memo_report); }
  const int z = d->width == 4 ? 0 : d->width == 8 ? 1 : d->width == 16 ? 2 : 3, n = d->width * d->width;
  memo_calls[z]++;
  for (int k = 0; k < MEMO_KS; k++) {
    int hit = 0;
    for (int i = 0; i < memo_k[k] && !hit; i++) {
      const memo_e *m = &memo[k][i];
      hit = m->valid && m->w == d->width && m->comp == d->comp && m->scan == d->scan_type && m->ts == d->transform_skip &&
            !memcmp(m->coef, coef, 4 * n) && memo_same_ctx(m->st, st, d->comp ? 1 : 0);
    }
    if (hit) { memo_hits[k][z]++; continue; }
    memo_e *m = &memo[k][memo_pos[k]];
    memo_pos[k] = (memo_pos[k] + 1) % memo_k[k];
    m->valid = 1; m->w = d->width; m->comp = d->comp; m->scan = d->scan_type; m->ts = d->transform_skip;
    memcpy(m->coef, coef, 4 * n); memcpy(m->st, st, 202);
  }
}
#endif
static void code_coeff_nxn(hm_enc *e, const hm_cu *cu, const tu_t *t, int comp, const int32_t *coef) {
  hvx_tu_desc d;
  tu_desc(e, cu, t, comp, &d);
#ifdef HVXO_MEMO_STATS
  memo_probe(&d, coef, e->cur->st);
#endif
  hvx_coeff_bits o;
  hvxo_coeff_bits(&d, coef, e->cur->st, e->pic->entropy_bits, &o);
  e->cur->frac += o.frac_bits;
}
/* TEncEntropy::estimateBit (TEncEntropy.cpp:685) from the current coder */
static void estimate_bit(hm_enc *e, int w, int h, int ch) {
  static const uint32_t rice[4] = {0, 0, 0, 0};
  hvxo_estbits_update(e->cur->st, e->pic->entropy_bits, rice, w, h, ch, &e->est);
}

/* ============================================================================================
 * xEncodeTransform (TEncEntropy.cpp:200) and encodeCoeff (:615) on the CU's coefficients
 * ========================================================================================== */
static void encode_transform(hm_enc *e, const hm_cu *cu, const tu_t *t) {
  const int rel = tu_abs_rel(t);
  const int trd = tu_depth_rel(t);
  const int subdiv = cu->p[rel].tr_idx > trd;
  const int l2 = t->log2;
  int cbf[3], any = 0;
  for (int c = 0; c < 3; c++) { cbf[c] = cbf_at(&cu->p[rel], c, trd); any |= cbf[c]; }
  const int intra = cu->p[rel].pred == MODE_INTRA;
  if (intra && cu->p[rel].part == SIZE_NxN && trd == 0) { /* inferred split */
  } else if (l2 > 5) {
  } else if (l2 == 2) {
  } else if (l2 == qt_min_log2(cu, rel)) {
  } else code_subdiv(e, subdiv, 5 - l2);
  const int first = trd == 0;
  for (int c = 1; c < 3; c++) {
    if (first || t->all[c]) {
      if (first || cbf_at(&cu->p[rel], c, trd - 1)) code_qt_cbf(e, cu, t, c, !subdiv);
    }
  }
  if (subdiv) {
    tu_t ch;
    tu_child(&ch, t, 1);
    do encode_transform(e, cu, &ch); while (tu_next(&ch, t));
    return;
  }
  if (!intra && trd == 0 && !cbf_at(&cu->p[rel], 1, 0) && !cbf_at(&cu->p[rel], 2, 0)) {
    /* luma cbf inferred */
  } else code_qt_cbf(e, cu, t, 0, 1);
  if (any)
    for (int c = 0; c < 3; c++)
      if (tu_proc(t, c) && cbf[c]) code_coeff_nxn(e, cu, t, c, cu->coef[c] + t->off[c]);
}
static void encode_coeff(hm_enc *e, const hm_cu *cu, int rel) {
  if (cu->p[rel].pred != MODE_INTRA) {
    if (!(cu->p[rel].merge && cu->p[rel].part == SIZE_2Nx2N)) cbin(e, X_ROOT_CBF, cu_qt_root_cbf(cu, rel));
    if (!cu_qt_root_cbf(cu, rel)) return;
  }
  tu_t t;
  tu_root(&t, cu, 0);
  encode_transform(e, cu, &t);
}

/* ============================================================================================
 * Samples: originals, reference planes, reconstruction
 * ========================================================================================== */
static void copy_org_to_yuv(hm_enc *e, yuv_t *dst, const hm_cu *cu) { /* copyFromPicYuv */
  for (int c = 0; c < 3; c++) {
    const int s = c ? 1 : 0, n = cu->width >> s;
    const int x0 = cu->x >> s, y0 = cu->y >> s, W = e->pic->w >> s, H = e->pic->h >> s;
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++) {
        const int px = x0 + x, py = y0 + y;
        yaddr(dst, c, 0, 0)[y * ystride(c) + x] = (px < W && py < H) ? e->pic->org[c][py * e->pic->org_stride[c] + px] : 0;
      }
  }
}
/* the picture reconstruction: TComPicYuv rec of the current picture (read outside the picture
 * only through availability-masked intra neighbours) */
static int16_t *rec_at(hm_enc *e, int c, int x, int y) { return e->rec[c] + y * e->rs[c] + x; }

/* xCopyYuv2Pic (TEncCu.cpp:1514): the CU's part of a yuv buffer into the picture */
static void yuv_to_pic(hm_enc *e, yuv_t *src, const hm_cu *cu) {
  for (int c = 0; c < 3; c++) {
    const int s = c ? 1 : 0, n = cu->width >> s, x0 = cu->x >> s, y0 = cu->y >> s;
    const int W = e->pic->w >> s, H = e->pic->h >> s;
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++)
        if (x0 + x < W + 8 && y0 + y < H + 8) *rec_at(e, c, x0 + x, y0 + y) = yaddr(src, c, 0, 0)[y * ystride(c) + x];
  }
}
static void yuv_to_pic_comp(hm_enc *e, yuv_t *src, const hm_cu *cu, int c) {
  const int s = c ? 1 : 0, n = cu->width >> s, x0 = cu->x >> s, y0 = cu->y >> s;
  const int W = e->pic->w >> s, H = e->pic->h >> s;
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++)
      if (x0 + x < W + 8 && y0 + y < H + 8) *rec_at(e, c, x0 + x, y0 + y) = yaddr(src, c, 0, 0)[y * ystride(c) + x];
}
/* xCopyYuv2Tmp (TEncCu.cpp:1541): the child's best reconstruction into the parent's temp */
static void yuv_child_to_parent(yuv_t *dst, yuv_t *src, int idx, int child_w) {
  for (int c = 0; c < 3; c++) {
    const int s = c ? 1 : 0, n = child_w >> s, ox = (idx & 1) * n, oy = (idx >> 1) * n;
    for (int y = 0; y < n; y++)
      memcpy(yaddr(dst, c, ox, oy + y), yaddr(src, c, 0, y), sizeof(int16_t) * n);
  }
}

/* ============================================================================================
 * Motion compensation: TComPrediction::motionCompensation (TComPrediction.cpp:517) for one PU
 * into a yuv buffer at the PU's position in the CU.
 * ========================================================================================== */
static void mc_pu(hm_enc *e, const hm_cu *cu, int ps, int pu, int list /* -1: REF_PIC_LIST_X */, yuv_t *dst) {
  const hvxo_hm_pic *P = e->pic;
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, &a, &w, &h);
  part_position(cu, ps, pu, &xp, &yp, &w, &h);
  const hm_part *p = &cu->p[a];
  hvx_mc_job j;
  memset(&j, 0, sizeof(j));
  j.pic_w = P->w; j.pic_h = P->h; j.max_cu = 64;
  j.cu_x = cu->x; j.cu_y = cu->y;
  j.pu_x = xp; j.pu_y = yp; j.w = w; j.h = h;
  for (int l = 0; l < 2; l++) {
    const int use = list < 0 ? p->ref[l] >= 0 : (l == list);
    j.ref[l] = use ? P->ref_plane_idx[l][p->ref[l]] : -1;
    j.poc[l] = use ? P->ref_poc[l][p->ref[l]] : 0;
    j.mv_x[l] = p->mv[l][0];
    j.mv_y[l] = p->mv[l][1];
  }
  j.flags = P->slice_type == B_SLICE ? HVX_MC_B_SLICE : 0;
  static _Thread_local int16_t out[64 * 64 + 2 * 32 * 32];
  hvxo_mc(P->ref_planes16, P->ref_stride16[0], P->ref_stride16[1], &j, out);
  const int rx = xp - cu->x, ry = yp - cu->y;
  for (int y = 0; y < h; y++) memcpy(yaddr(dst, 0, rx, ry + y), out + y * w, sizeof(int16_t) * w);
  for (int c = 1; c < 3; c++)
    for (int y = 0; y < (h >> 1); y++)
      memcpy(yaddr(dst, c, rx >> 1, (ry >> 1) + y), out + w * h + (c - 1) * (w >> 1) * (h >> 1) + y * (w >> 1),
             sizeof(int16_t) * (w >> 1));
}
static void mc_cu(hm_enc *e, const hm_cu *cu, yuv_t *dst) {
  const int ps = cu->p[0].part;
  for (int pu = 0; pu < num_parts_of(ps); pu++) mc_pu(e, cu, ps, pu, -1, dst);
}

/* ============================================================================================
 * Merge candidates: TComDataCU::getInterMergeCandidates (TComDataCU.cpp:2182) with
 * xGetColMVP (:3061), xGetDistScaleFactor (:3133), hasEqualMotion (:2159); P and B slices.
 * ========================================================================================== */
typedef struct { int16_t mv[2]; int ref; } mvfield_t;

static int dist_scale(int cur_poc, int cur_ref_poc, int col_poc, int col_ref_poc) {
  const int dd = col_poc - col_ref_poc, db = cur_poc - cur_ref_poc;
  if (dd == db) return 4096;
  const int tb = db < -128 ? -128 : db > 127 ? 127 : db, td = dd < -128 ? -128 : dd > 127 ? 127 : dd;
  const int x = (0x4000 + abs(td / 2)) / td;
  int s = (tb * x + 32) >> 6;
  return s < -4096 ? -4096 : s > 4095 ? 4095 : s;
}
static int16_t scale_comp(int s, int v) {
  int r = (s * v + 127 + (s * v < 0)) >> 8;
  return (int16_t)(r < -32768 ? -32768 : r > 32767 ? 32767 : r);
}
/* xGetColMVP: the collocated partition (ctu, z) of the col picture's compressed field */
static int col_mvp(const hm_enc *e, int list, int ctu, int z, int ref_idx, int16_t *mv) {
  const hvxo_hm_pic *P = e->pic;
  if (!P->col_valid) return 0;
  const int16_t *f = P->col_field + ((size_t)ctu * 16 + (z >> 4)) * 8;
  if (f[0] != MODE_INTER) return 0;
  int cl = P->check_ldc ? list : P->col_from_l0;
  int cr = f[1 + cl];
  if (cr < 0) {
    cl = 1 - cl;
    cr = f[1 + cl];
    if (cr < 0) return 0;
  }
  const int col_ref_poc = P->col_ref_poc[cl][cr];
  const int cmx = f[3 + 2 * cl], cmy = f[4 + 2 * cl];
  const int cur_ref_poc = P->ref_poc[list][ref_idx];
  const int s = dist_scale(P->poc, cur_ref_poc, P->col_poc, col_ref_poc);
  if (s == 4096) { mv[0] = (int16_t)cmx; mv[1] = (int16_t)cmy; }
  else { mv[0] = scale_comp(s, cmx); mv[1] = scale_comp(s, cmy); }
  return 1;
}
/* the TMVP bottom-right / centre positions (:2370-2420, :2714-2755) */
static void col_positions(const hm_enc *e, const hm_cu *cu, int ps, int pu, int *br_ctu, int *br_z, int *c_z) {
  const int rb = pu_right_bottom(cu, ps, pu), r = Z2R[rb];
  *br_ctu = -1;
  *br_z = 0;
  if (e->ctu_x * 64 + RPX(r) + 4 < e->pic->w && e->ctu_y * 64 + RPY(r) + 4 < e->pic->h) {
    if ((r & 15) < 15 && (r >> 4) < 15) { *br_z = R2Z[r + 17]; *br_ctu = e->ctu_addr; }
    else if ((r & 15) < 15) { *br_z = R2Z[(r + 17) % 256]; }
    else if ((r >> 4) < 15) { *br_z = R2Z[r + 1]; *br_ctu = e->ctu_addr + 1; }
    else *br_z = 0;
  }
  *c_z = pu_center(cu, ps, pu);
}
static int same_motion(const hm_part *a, const hm_part *b) {
  if (a->inter_dir != b->inter_dir) return 0;
  for (int l = 0; l < 2; l++)
    if (a->inter_dir & (1 << l))
      if (a->mv[l][0] != b->mv[l][0] || a->mv[l][1] != b->mv[l][1] || a->ref[l] != b->ref[l]) return 0;
  return 1;
}
static void nb_field(nb_t n, int list, mvfield_t *f) {
  f->mv[0] = n.p[n.idx].mv[list][0];
  f->mv[1] = n.p[n.idx].mv[list][1];
  f->ref = n.p[n.idx].ref[list];
}
static int merge_candidates(const hm_enc *e, const hm_cu *cu, int ps, int pu, mvfield_t *f /* [2*5] */, int *dirs) {
  const hvxo_hm_pic *P = e->pic;
  const int maxc = P->max_merge, isb = P->slice_type == B_SLICE;
  int is_inter[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < maxc; i++) { f[2 * i].ref = -1; f[2 * i + 1].ref = -1; f[2 * i].mv[0] = f[2 * i].mv[1] = 0; f[2 * i + 1].mv[0] = f[2 * i + 1].mv[1] = 0; dirs[i] = 0; }
  int lt, rt, lb;
  pu_corners(cu, ps, pu, &lt, &rt, &lb);
  int cnt = 0;
  /* A1 */
  nb_t l = get_pu_left(e, cu, lb);
  const int a1 = l.valid && !(pu == 1 && (ps == SIZE_Nx2N || ps == SIZE_nLx2N || ps == SIZE_nRx2N)) && nb_inter(l);
  if (a1) {
    is_inter[cnt] = 1; dirs[cnt] = l.p[l.idx].inter_dir;
    nb_field(l, 0, &f[2 * cnt]);
    if (isb) nb_field(l, 1, &f[2 * cnt + 1]);
    cnt++;
  }
  if (cnt == maxc) return cnt;
  /* B1 */
  nb_t a = get_pu_above(e, cu, rt, 0);
  const int b1 = a.valid && !(pu == 1 && (ps == SIZE_2NxN || ps == SIZE_2NxnU || ps == SIZE_2NxnD)) && nb_inter(a);
  if (b1 && (!a1 || !same_motion(&l.p[l.idx], &a.p[a.idx]))) {
    is_inter[cnt] = 1; dirs[cnt] = a.p[a.idx].inter_dir;
    nb_field(a, 0, &f[2 * cnt]);
    if (isb) nb_field(a, 1, &f[2 * cnt + 1]);
    cnt++;
  }
  if (cnt == maxc) return cnt;
  /* B0 */
  nb_t ar = get_pu_above_right(e, cu, rt, 1);
  const int b0 = nb_inter(ar);
  if (b0 && (!b1 || !same_motion(&a.p[a.idx], &ar.p[ar.idx]))) {
    is_inter[cnt] = 1; dirs[cnt] = ar.p[ar.idx].inter_dir;
    nb_field(ar, 0, &f[2 * cnt]);
    if (isb) nb_field(ar, 1, &f[2 * cnt + 1]);
    cnt++;
  }
  if (cnt == maxc) return cnt;
  /* A0 */
  nb_t bl = get_pu_below_left(e, cu, lb, 1);
  const int a0 = nb_inter(bl);
  if (a0 && (!a1 || !same_motion(&l.p[l.idx], &bl.p[bl.idx]))) {
    is_inter[cnt] = 1; dirs[cnt] = bl.p[bl.idx].inter_dir;
    nb_field(bl, 0, &f[2 * cnt]);
    if (isb) nb_field(bl, 1, &f[2 * cnt + 1]);
    cnt++;
  }
  if (cnt == maxc) return cnt;
  /* B2 */
  if (cnt < 4) {
    int a_off, w, h;
    part_index_size(cu, ps, pu, &a_off, &w, &h);
    nb_t al = get_pu_above_left(e, cu, cu->zidx + a_off);
    const int b2 = nb_inter(al);
    if (b2 && (!a1 || !same_motion(&l.p[l.idx], &al.p[al.idx])) && (!b1 || !same_motion(&a.p[a.idx], &al.p[al.idx]))) {
      is_inter[cnt] = 1; dirs[cnt] = al.p[al.idx].inter_dir;
      nb_field(al, 0, &f[2 * cnt]);
      if (isb) nb_field(al, 1, &f[2 * cnt + 1]);
      cnt++;
    }
  }
  if (cnt == maxc) return cnt;
  /* temporal */
  if (P->tmvp) {
    int br_ctu, br_z, c_z, dir = 0;
    col_positions(e, cu, ps, pu, &br_ctu, &br_z, &c_z);
    int16_t mv[2];
    int ex = br_ctu >= 0 && col_mvp(e, 0, br_ctu, br_z, 0, mv);
    if (!ex) ex = col_mvp(e, 0, e->ctu_addr, c_z, 0, mv);
    if (ex) { dir |= 1; f[2 * cnt].mv[0] = mv[0]; f[2 * cnt].mv[1] = mv[1]; f[2 * cnt].ref = 0; }
    if (isb) {
      ex = br_ctu >= 0 && col_mvp(e, 1, br_ctu, br_z, 0, mv);
      if (!ex) ex = col_mvp(e, 1, e->ctu_addr, c_z, 0, mv);
      if (ex) { dir |= 2; f[2 * cnt + 1].mv[0] = mv[0]; f[2 * cnt + 1].mv[1] = mv[1]; f[2 * cnt + 1].ref = 0; }
    }
    if (dir) { dirs[cnt] = dir; is_inter[cnt] = 1; cnt++; }
  }
  if (cnt == maxc) return cnt;
  int arr = cnt;
  const int cutoff = arr;
  if (isb) {
    static const int l0[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3}, l1[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};
    for (int idx = 0; idx < cutoff * (cutoff - 1) && arr != maxc; idx++) {
      const int i = l0[idx], j = l1[idx];
      if (is_inter[i] && is_inter[j] && (dirs[i] & 1) && (dirs[j] & 2)) {
        is_inter[arr] = 1;
        dirs[arr] = 3;
        f[2 * arr] = f[2 * i];
        f[2 * arr + 1] = f[2 * j + 1];
        const int p0 = P->ref_poc[0][f[2 * arr].ref], p1 = P->ref_poc[1][f[2 * arr + 1].ref];
        if (p0 == p1 && f[2 * arr].mv[0] == f[2 * arr + 1].mv[0] && f[2 * arr].mv[1] == f[2 * arr + 1].mv[1]) is_inter[arr] = 0;
        else arr++;
      }
    }
  }
  if (arr == maxc) return arr;
  const int nref = isb ? (P->nref[0] < P->nref[1] ? P->nref[0] : P->nref[1]) : P->nref[0];
  int r = 0, refcnt = 0;
  while (arr < maxc) {
    is_inter[arr] = 1;
    dirs[arr] = 1;
    f[2 * arr].mv[0] = f[2 * arr].mv[1] = 0; f[2 * arr].ref = r;
    if (isb) { dirs[arr] = 3; f[2 * arr + 1].mv[0] = f[2 * arr + 1].mv[1] = 0; f[2 * arr + 1].ref = r; }
    arr++;
    if (refcnt == nref - 1) r = 0;
    else { r++; refcnt++; }
  }
  return arr;
}

/* ============================================================================================
 * AMVP: fillMvpCand (TComDataCU.cpp:2623) with xAddMVPCand (:2850) / xAddMVPCandOrder (:2936)
 * ========================================================================================== */
typedef struct { int n; int16_t c[3][2]; } amvp_t;

static int add_mvp(const hm_enc *e, amvp_t *in, int list, int ref_idx, nb_t n) {
  const hvxo_hm_pic *P = e->pic;
  if (!n.valid) return 0;
  const hm_part *q = &n.p[n.idx];
  const int cur_ref_poc = P->ref_poc[list][ref_idx];
  if (q->ref[list] >= 0 && cur_ref_poc == P->ref_poc[list][q->ref[list]]) {
    in->c[in->n][0] = q->mv[list][0]; in->c[in->n][1] = q->mv[list][1]; in->n++;
    return 1;
  }
  const int l2 = 1 - list;
  if (q->ref[l2] >= 0 && P->ref_poc[l2][q->ref[l2]] == cur_ref_poc) {
    in->c[in->n][0] = q->mv[l2][0]; in->c[in->n][1] = q->mv[l2][1]; in->n++;
    return 1;
  }
  return 0;
}
static int add_mvp_order(const hm_enc *e, amvp_t *in, int list, int ref_idx, nb_t n) {
  const hvxo_hm_pic *P = e->pic;
  if (!n.valid) return 0;
  const hm_part *q = &n.p[n.idx];
  const int cur_ref_poc = P->ref_poc[list][ref_idx];
  for (int k = 0; k < 2; k++) {
    const int ll = k ? 1 - list : list;
    if (q->ref[ll] >= 0) {
      const int nrp = P->ref_poc[ll][q->ref[ll]];
      const int s = dist_scale(P->poc, cur_ref_poc, P->poc, nrp);
      if (s == 4096) { in->c[in->n][0] = q->mv[ll][0]; in->c[in->n][1] = q->mv[ll][1]; }
      else { in->c[in->n][0] = scale_comp(s, q->mv[ll][0]); in->c[in->n][1] = scale_comp(s, q->mv[ll][1]); }
      in->n++;
      return 1;
    }
  }
  return 0;
}
static void fill_mvp_cand(const hm_enc *e, const hm_cu *cu, int ps, int pu, int list, int ref_idx, amvp_t *in) {
  in->n = 0;
  int lt, rt, lb;
  pu_corners(cu, ps, pu, &lt, &rt, &lb);
  nb_t bl = get_pu_below_left(e, cu, lb, 1);
  int added_smvp = nb_inter(bl);
  nb_t l = get_pu_left(e, cu, lb);
  if (!added_smvp) added_smvp = nb_inter(l);
  int added = add_mvp(e, in, list, ref_idx, bl);
  if (!added) added = add_mvp(e, in, list, ref_idx, l);
  if (!added) {
    added = add_mvp_order(e, in, list, ref_idx, bl);
    if (!added) add_mvp_order(e, in, list, ref_idx, l);
  }
  nb_t ar = get_pu_above_right(e, cu, rt, 1), a = get_pu_above(e, cu, rt, 0), al = get_pu_above_left(e, cu, lt);
  added = add_mvp(e, in, list, ref_idx, ar);
  if (!added) added = add_mvp(e, in, list, ref_idx, a);
  if (!added) add_mvp(e, in, list, ref_idx, al);
  if (!added_smvp) {
    added = add_mvp_order(e, in, list, ref_idx, ar);
    if (!added) added = add_mvp_order(e, in, list, ref_idx, a);
    if (!added) add_mvp_order(e, in, list, ref_idx, al);
  }
  if (in->n == 2 && in->c[0][0] == in->c[1][0] && in->c[0][1] == in->c[1][1]) in->n = 1;
  if (e->pic->tmvp) {
    int br_ctu, br_z, c_z;
    col_positions(e, cu, ps, pu, &br_ctu, &br_z, &c_z);
    int16_t mv[2];
    if ((br_ctu >= 0 && col_mvp(e, list, br_ctu, br_z, ref_idx, mv)) || col_mvp(e, list, e->ctu_addr, c_z, ref_idx, mv)) {
      in->c[in->n][0] = mv[0]; in->c[in->n][1] = mv[1]; in->n++;
    }
  }
  if (in->n > 2) in->n = 2;
  while (in->n < 2) { in->c[in->n][0] = in->c[in->n][1] = 0; in->n++; }
}

/* ============================================================================================
 * TComRdCost: calcRdCost (TComRdCost.cpp:57), getCost (TComRdCost.h:183), getDistPart (:429)
 * ========================================================================================== */
static double rd_cost(const hm_enc *e, uint32_t bits, uint32_t dist) {
  return floor((double)dist + (double)bits * e->pic->lambda + 0.5);
}
static double rd_cost_sad(const hm_enc *e, uint32_t bits, uint32_t dist) {
  return floor((double)dist + (floor((double)bits * (double)e->pic->lambda_motion + 0.5) / 65536.0));
}
/* The SSIM RD cost of the CU decision (hvx_hm_picture.rd_metric = HVX_RD_SSIM; the stvssim JM
 * encoder's mode-decision cost, rdopt.c:1631 J = D + lambda * max(0.5, R) with D = 1 - SSIM per
 * component, distortionSSIM stvssim.c:567-584, and lambda = lambda_2(QP) * eta^0.85, stvssim.c:1805,
 * :1707), adapted to HEVC CUs: D of a CU = sum over its 8x8 luma blocks of (1 - SSIM) (one 8x8
 * window, compute_SSIM stvssim.c:491-566) plus over its 4x4 Cb and Cr blocks (one 4x4 window),
 * each term weighted 1/4 so that a 16x16 area weighs as one JM macroblock; blocks outside the
 * picture are skipped; the terms are summed in double, luma blocks in raster order, then Cb, Cr.
 * Only TEncCu's mode and split comparisons use it (xCheckBestMode :1444 and the split cost); the
 * searches, merge estimation, RQT and RDOQ below keep HM's SSE / SATD costs. */
/* one block, one window: compute_SSIM through the pinned hvxo_ssim (tests/golden/ssim.bin) */
static float ssim_block16(const int16_t *o, const int16_t *r, int stride, int wint) {
  uint8_t o8[64], r8[64];
  for (int y = 0; y < wint; y++)
    for (int x = 0; x < wint; x++) { o8[y * wint + x] = (uint8_t)o[y * stride + x]; r8[y * wint + x] = (uint8_t)r[y * stride + x]; }
  return hvxo_ssim(o8, wint, r8, wint, wint, wint, wint, wint);
}
static double cu_dssim(const hm_enc *e, const hm_cu *cu, yuv_t *org, yuv_t *reco) {
  const hvxo_hm_pic *P = e->pic;
  double d = 0;
  for (int c = 0; c < 3; c++) {
    const int s = c ? 1 : 0, b = c ? 4 : 8, n = (cu->width >> s) / b;
    for (int by = 0; by < n; by++)
      for (int bx = 0; bx < n; bx++) {
        if (((cu->x >> s) + bx * b) >= (P->w >> s) || ((cu->y >> s) + by * b) >= (P->h >> s)) continue;
        const float v = ssim_block16(yaddr(org, c, bx * b, by * b), yaddr(reco, c, bx * b, by * b), ystride(c), b);
        d += 0.25 * (double)(1.0f - v);
      }
  }
  return d;
}
/* The stVSSIM RD cost (rd_metric 2 = HVX_RD_STVSSIM; include/hvx_types.h hvx_hm_picture.hist): the
 * stvssim encoder's active distortion, distortionstVSSIM (stvssim.c:831-855, att_stv.h:5, rdopt.c:223),
 * per JM macroblock -- a 16x16 luma area of the CU with its 8x8 Cb, Cr blocks, in raster order --
 * D_mb = (1 - stVSSIM_Y) * WeightY + (1 - stVSSIM_Cb) * WeightCb + (1 - stVSSIM_Cr) * WeightCr, the
 * weights 1 (encoder.cfg:289-291) in double, and stVSSIM = compute_stVSSIM's stvssimValue (:587-830:
 * 8x8 windows stepped by SSIMOverlapSize 4, encoder.cfg:280) over hist_n + 1 frames (the history, most
 * recent first, then the CU's own original / reconstruction), through the pinned hvxo_stvssim
 * (tests/golden/ssim.bin).  Cr reads Cb's history planes: compute_stVSSIM is called with comp 1 for
 * both chroma components (:846, :850).  An 8x8 CU (smaller than a macroblock) is one 8x8 luma window
 * and 4x4 chroma windows (compute_stVSSIM's wint 4 filters), weighted 1/4. */
static float stv_term(const hm_enc *e, yuv_t *org, yuv_t *reco, int c, int lx, int ly, int px, int py, int bw, int wint) {
  const hvxo_hm_pic *P = e->pic;
  const int used = P->hist_n + 1, hc = c == 2 ? 1 : c, s = c ? 1 : 0, uv = c ? 2 : 1, dw = bw * uv;
  static __thread uint8_t ob[26][256], rb[26][256];
  static __thread float dm[32 * 32];
  const uint8_t *op[26], *rp[26];
  for (int o = 0; o < used; o++) {
    for (int y = 0; y < bw; y++)
      for (int x = 0; x < bw; x++) {
        if (o < used - 1) {
          const int st = P->hist_stride[s];
          ob[o][y * bw + x] = P->hist[6 * o + hc][(py + y) * st + px + x];
          rb[o][y * bw + x] = P->hist[6 * o + 3 + hc][(py + y) * st + px + x];
        } else {
          ob[o][y * bw + x] = (uint8_t)yaddr(org, c, lx, ly)[y * ystride(c) + x];
          rb[o][y * bw + x] = (uint8_t)yaddr(reco, c, lx, ly)[y * ystride(c) + x];
        }
      }
    op[o] = ob[o];
    rp[o] = rb[o];
  }
  for (int y = 0; y < dw; y++)
    for (int x = 0; x < dw; x++)
      dm[y * dw + x] = P->dirs ? P->dirs[((py * uv + y) >> 2) * P->dirs_stride + ((px * uv + x) >> 2)] : 0.0f;
  float ss, s3, stv;
  hvxo_stvssim(op, rp, bw, dm, dw, bw, bw, wint, 4, used, c ? 1 : 0, &ss, &s3, &stv);
  return 1.0f - stv;
}
static double cu_dstv(const hm_enc *e, const hm_cu *cu, yuv_t *org, yuv_t *reco) {
  const hvxo_hm_pic *P = e->pic;
  if (cu->width == 8) {
    const float dy = stv_term(e, org, reco, 0, 0, 0, cu->x, cu->y, 8, 8);
    const float du = stv_term(e, org, reco, 1, 0, 0, cu->x >> 1, cu->y >> 1, 4, 4);
    const float dv = stv_term(e, org, reco, 2, 0, 0, cu->x >> 1, cu->y >> 1, 4, 4);
    return 0.25 * ((double)dy * 1.0 + (double)du * 1.0 + (double)dv * 1.0);
  }
  const int n = cu->width >> 4;
  double d = 0;
  for (int my = 0; my < n; my++)
    for (int mx = 0; mx < n; mx++) {
      const int x = cu->x + 16 * mx, y = cu->y + 16 * my;
      if (x >= P->w || y >= P->h) continue;
      const float dy = stv_term(e, org, reco, 0, 16 * mx, 16 * my, x, y, 16, 8);
      const float du = stv_term(e, org, reco, 1, 8 * mx, 8 * my, x >> 1, y >> 1, 8, 8);
      const float dv = stv_term(e, org, reco, 2, 8 * mx, 8 * my, x >> 1, y >> 1, 8, 8);
      d += (double)dy * 1.0 + (double)du * 1.0 + (double)dv * 1.0;
    }
  return d;
}
/* the cost TEncCu compares: calcRdCost(bits, dist) (SSE) or the SSIM / stVSSIM cost */
static double cu_cost(const hm_enc *e, const hm_cu *cu, uint32_t bits, uint32_t dist) {
  if (e->pic->rd_metric == 0) return rd_cost(e, bits, dist);
  return cu->dssim + e->pic->lambda_ssim * ((double)bits > 0.5 ? (double)bits : 0.5);
}
static void cu_measure_ssim(const hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *reco) {
  if (e->pic->rd_metric == 1) cu->dssim = cu_dssim(e, cu, org, reco);
  else if (e->pic->rd_metric == 2) cu->dssim = cu_dstv(e, cu, org, reco);
}
static uint32_t mv_cost_bits(const hm_enc *e, uint32_t bits) { return (uint32_t)(e->pic->lambda_motion * bits) >> 16; }
static uint32_t dist_part(const hm_enc *e, const int16_t *a, int sa, const int16_t *b, int sb, int w, int h, int comp) {
  const uint32_t sse = hvxo_sse(a, sa, b, sb, w, h);
  if (comp) return (uint32_t)(e->pic->chroma_weight[comp - 1] * (double)sse);
  return sse;
}

/* ============================================================================================
 * Inter residual: encodeResAndCalcRdInterCU (TEncSearch.cpp:4280) with xEstimateInterResidualQT
 * (:4426), xEncodeInterResidualQT (:5069), xSetInterResidualQTData (:5157), xAddSymbolBitsInter
 * (:5290).  Residual and QT buffers are addressed relative to the CU.
 * ========================================================================================== */
static int qt_layer(int log2) { return 5 - log2; }
static void set_cbf_range(hm_cu *cu, int comp, int rel, int n, int v) { for (int i = 0; i < n; i++) cu->p[rel + i].cbf[comp] = (uint8_t)v; }

static void transform_tu(hm_enc *e, const hm_cu *cu, const tu_t *t, int comp, const int16_t *resi, int rs, int32_t *coef,
                         int32_t *abs_sum) {
  hvx_tu_desc d;
  tu_desc(e, cu, t, comp, &d);
  int32_t tmp[1024], arl[1024];
  hvxo_transform_nxn(&d, &e->est, resi, rs, tmp, coef, arl, abs_sum);
  /* transformNxN sets the CBF byte of the TU (TComTrQuant.cpp:1543): GetAbsPartIdxTU() over
   * GetAbsPartIdxNumParts(compID), at the luma transform depth */
  set_cbf_range((hm_cu *)cu, comp, tu_abs_rel(t), tu_nparts(t, comp), (*abs_sum > 0 ? 1 : 0) << tu_depth_rel(t));
}
static void inv_transform_tu(hm_enc *e, const hm_cu *cu, const tu_t *t, int comp, const int32_t *coef, int16_t *resi, int rs) {
  hvx_tu_desc d;
  tu_desc(e, cu, t, comp, &d);
  hvxo_inv_transform_nxn(&d, coef, resi, rs);
}
static void set_ts_range(hm_cu *cu, int comp, int rel, int n, int v) { for (int i = 0; i < n; i++) cu->p[rel + i].ts[comp] = (uint8_t)v; }
static void set_tridx(hm_cu *cu, int rel, int n, int v) { for (int i = 0; i < n; i++) cu->p[rel + i].tr_idx = (int8_t)v; }

static void encode_inter_residual_qt(hm_enc *e, const hm_cu *cu, int comp /* 3: cbfs */, const tu_t *t);

static void estimate_inter_residual_qt(hm_enc *e, hm_cu *cu, yuv_t *resi, double *rd, uint32_t *bits, uint32_t *dist,
                                       uint32_t *zero_dist, const tu_t *t) {
  const int rel = tu_abs_rel(t), depth = tu_depth_total(t), trmode = tu_depth_rel(t), l2 = t->log2;
  const int check_full = l2 <= 5;
  const int check_split = l2 > qt_min_log2(cu, rel);
  double single_cost = MAX_DOUBLE;
  uint32_t single_bits = 0, single_dist = 0;
  uint32_t single_dist_comp[3] = {0, 0, 0};
  int32_t abs_sum[3] = {0, 0, 0};
  int best_mode[3] = {0, 0, 0};
  const int layer = qt_layer(l2);
  load(&e->rd[depth][CI_QT_TRAFO_ROOT], e->cur);
  if (check_full) {
    double min_cost[3] = {MAX_DOUBLE, MAX_DOUBLE, MAX_DOUBLE};
    set_tridx(cu, rel, t->step, trmode);
    reset_bits(e);
    for (int comp = 0; comp < 3; comp++) {
      if (!tu_proc(t, comp)) continue;
      const int crel = tu_abs_rel_c(t, comp), np = tu_nparts(t, comp);
      const int w = t->w[comp], h = t->h[comp], x0 = t->x0[comp], y0 = t->y0[comp];
      const int check_ts = w <= 4; /* TransformSkip on, TUCompRectHasAssociatedTransformSkipFlag (log2 max 2) */
      int32_t *cur_coef = e->qt_coef[comp][layer] + t->off[comp];
      int16_t *qres = yaddr(&e->qt_yuv[layer], comp, x0, y0);
      const int qs = ystride(comp);
      int16_t *pres = yaddr(resi, comp, x0, y0);
      const int modes = check_ts ? 2 : 1;
      for (int mode = 0; mode < modes; mode++) {
        const int first = mode == 0;
        set_ts_range(cu, comp, crel, np, mode);
        load(e->cur, &e->rd[depth][CI_QT_TRAFO_ROOT]);
        reset_bits(e);
        set_ts_range(cu, comp, crel, np, mode);
        if (comp != 2) estimate_bit(e, w, h, comp ? 1 : 0);
        int32_t best_coef[1024];
        int16_t best_res[1024];
        int32_t cur_abs = 0;
        uint32_t cur_bits = 0, cur_dist = 0, non_bits = 0, non_dist = 0;
        double cur_cost = 0, non_cost = 0;
        if (!first) {
          memcpy(best_coef, cur_coef, sizeof(int32_t) * w * h);
          for (int y = 0; y < h; y++) memcpy(&best_res[y * w], qres + y * qs, sizeof(int16_t) * w);
        }
        transform_tu(e, cu, t, comp, pres, ystride(comp), cur_coef, &cur_abs);
        if (first || cur_abs == 0) {
          int16_t zero[1024];
          memset(zero, 0, sizeof(zero));
          non_dist = dist_part(e, zero, w, pres, ystride(comp), w, h, comp);
          code_qt_cbf_zero(e, t, comp ? 1 : 0);
          non_bits = written_bits(e);
          non_cost = rd_cost(e, non_bits, non_dist);
        }
        if (zero_dist && first) *zero_dist += non_dist;
        if (cur_abs > 0) {
          if (first) {
            load(e->cur, &e->rd[depth][CI_QT_TRAFO_ROOT]);
            reset_bits(e);
          }
          code_qt_cbf(e, cu, t, comp, 1); /* the CBF transformNxN just set */
          code_coeff_nxn(e, cu, t, comp, cur_coef);
          cur_bits = written_bits(e);
          inv_transform_tu(e, cu, t, comp, cur_coef, qres, qs);
          cur_dist = dist_part(e, qres, qs, pres, ystride(comp), w, h, comp);
          cur_cost = rd_cost(e, cur_bits, cur_dist);
        } else if (mode == 1) {
          cur_cost = MAX_DOUBLE;
        } else {
          cur_bits = non_bits; cur_dist = non_dist; cur_cost = non_cost;
        }
        if (cur_cost < min_cost[comp] || (mode == 1 && cur_cost == min_cost[comp])) {
          if (first && (non_cost < cur_cost || cur_abs == 0)) {
            memset(cur_coef, 0, sizeof(int32_t) * w * h);
            cur_abs = 0; cur_bits = non_bits; cur_dist = non_dist; cur_cost = non_cost;
          }
          abs_sum[comp] = cur_abs;
          single_dist_comp[comp] = cur_dist;
          min_cost[comp] = cur_cost;
          best_mode[comp] = mode;
          if (cur_abs == 0)
            for (int y = 0; y < h; y++) memset(qres + y * qs, 0, sizeof(int16_t) * w);
        } else {
          memcpy(cur_coef, best_coef, sizeof(int32_t) * w * h);
          for (int y = 0; y < h; y++) memcpy(qres + y * qs, &best_res[y * w], sizeof(int16_t) * w);
        }
        (void)cur_bits;
      }
      set_ts_range(cu, comp, crel, np, best_mode[comp]);
      set_cbf_range(cu, comp, crel, np, (abs_sum[comp] > 0 ? 1 : 0) << trmode);
    }
    load(e->cur, &e->rd[depth][CI_QT_TRAFO_ROOT]);
    reset_bits(e);
    if (l2 > qt_min_log2(cu, rel)) code_subdiv(e, 0, 5 - l2);
    for (int ch = 0; ch < 3; ch++) {
      const int comp = (ch + 1) == 3 ? 0 : ch + 1;
      if (tu_proc(t, comp)) code_qt_cbf(e, cu, t, comp, 1);
    }
    for (int comp = 0; comp < 3; comp++)
      if (tu_proc(t, comp)) {
        if (cbf_at(&cu->p[tu_abs_rel_c(t, comp)], comp, trmode))
          code_coeff_nxn(e, cu, t, comp, e->qt_coef[comp][layer] + t->off[comp]);
        single_dist += single_dist_comp[comp];
      }
    single_bits = written_bits(e);
    single_cost = rd_cost(e, single_bits, single_dist);
  }
  if (check_split) {
    if (check_full) {
      load(&e->rd[depth][CI_QT_TRAFO_TEST], e->cur);
      load(e->cur, &e->rd[depth][CI_QT_TRAFO_ROOT]);
    }
    uint32_t sub_dist = 0, sub_bits = 0;
    double sub_cost = 0;
    int best_cbf[3];
    for (int c = 0; c < 3; c++)
      if (tu_proc(t, c)) best_cbf[c] = cbf_at(&cu->p[rel], c, trmode);
    tu_t ch;
    tu_child(&ch, t, 0);
    const int qparts = ch.step;
    do estimate_inter_residual_qt(e, cu, resi, &sub_cost, &sub_bits, &sub_dist, check_full ? NULL : zero_dist, &ch);
    while (tu_next(&ch, t));
    int any = 0;
    for (int c = 0; c < 3; c++) {
      int yuv = 0;
      for (int i = 0; i < 4; i++) yuv |= cbf_at(&cu->p[rel + i * qparts], c, trmode + 1);
      for (int i = 0; i < 4 * qparts; i++) cu->p[rel + i].cbf[c] |= (uint8_t)(yuv << trmode);
      any |= yuv;
    }
    load(e->cur, &e->rd[depth][CI_QT_TRAFO_ROOT]);
    reset_bits(e);
    encode_inter_residual_qt(e, cu, 3, t);
    for (int c = 0; c < 3; c++) encode_inter_residual_qt(e, cu, c, t);
    sub_bits = written_bits(e);
    sub_cost = rd_cost(e, sub_bits, sub_dist);
    if (!check_full || (any && sub_cost < single_cost)) {
      *rd += sub_cost; *bits += sub_bits; *dist += sub_dist;
    } else {
      *rd += single_cost; *bits += single_bits; *dist += single_dist;
      set_tridx(cu, rel, t->step, trmode);
      for (int c = 0; c < 3; c++)
        if (tu_proc(t, c)) {
          const int crel = tu_abs_rel_c(t, c), np = tu_nparts(t, c);
          set_cbf_range(cu, c, crel, np, best_cbf[c] << trmode);
          set_ts_range(cu, c, crel, np, best_mode[c]);
        }
      load(e->cur, &e->rd[depth][CI_QT_TRAFO_TEST]);
    }
  } else {
    *rd += single_cost; *bits += single_bits; *dist += single_dist;
  }
}

static void encode_inter_residual_qt(hm_enc *e, const hm_cu *cu, int comp, const tu_t *t) {
  const int rel = tu_abs_rel(t), cur_tr = tu_depth_rel(t);
  const int trmode = cu->p[rel].tr_idx;
  const int subdiv = cur_tr != trmode;
  const int l2 = t->log2;
  if (comp == 3) {
    if (l2 <= 5 && l2 > qt_min_log2(cu, rel)) code_subdiv(e, subdiv, 5 - l2);
    const int first = cur_tr == 0;
    for (int c = 1; c < 3; c++) {
      if (first || t->all[c]) {
        if (first || cbf_at(&cu->p[rel], c, cur_tr - 1)) code_qt_cbf(e, cu, t, c, !subdiv);
      }
    }
    if (!subdiv) code_qt_cbf(e, cu, t, 0, 1);
  }
  if (!subdiv) {
    if (comp != 3 && tu_proc(t, comp)) {
      if (cbf_at(&cu->p[tu_abs_rel_c(t, comp)], comp, trmode))
        code_coeff_nxn(e, cu, t, comp, e->qt_coef[comp][qt_layer(l2)] + t->off[comp]);
    }
  } else {
    if (comp == 3 || cbf_at(&cu->p[rel], comp, cur_tr)) {
      tu_t ch;
      tu_child(&ch, t, 0);
      do encode_inter_residual_qt(e, cu, comp, &ch); while (tu_next(&ch, t));
    }
  }
}

/* xSetInterResidualQTData (:5157) */
static void set_inter_residual_qt_data(hm_enc *e, hm_cu *cu, yuv_t *resi, int spatial, const tu_t *t) {
  const int rel = tu_abs_rel(t);
  if (tu_depth_rel(t) == cu->p[rel].tr_idx) {
    const int layer = qt_layer(t->log2);
    for (int c = 0; c < 3; c++) {
      if (!tu_proc(t, c)) continue;
      const int w = t->w[c], h = t->h[c];
      if (spatial) {
        for (int y = 0; y < h; y++)
          memcpy(yaddr(resi, c, t->x0[c], t->y0[c] + y), yaddr(&e->qt_yuv[layer], c, t->x0[c], t->y0[c] + y), sizeof(int16_t) * w);
      } else {
        memcpy(cu->coef[c] + t->off[c], e->qt_coef[c][layer] + t->off[c], sizeof(int32_t) * w * h);
      }
    }
  } else {
    tu_t ch;
    tu_child(&ch, t, 0);
    do set_inter_residual_qt_data(e, cu, resi, spatial, &ch); while (tu_next(&ch, t));
  }
}

/* xAddSymbolBitsInter (:5290) */
static void add_symbol_bits_inter(hm_enc *e, hm_cu *cu, uint32_t *bits) {
  if (cu->p[0].merge && cu->p[0].part == SIZE_2Nx2N && !cu_qt_root_cbf(cu, 0)) {
    cu_set_all(cu, F_SKIP, 1);
    reset_bits(e);
    code_skip_flag(e, cu, 0);
    code_merge_index(e, cu, 0);
    *bits += written_bits(e);
  } else {
    reset_bits(e);
    code_skip_flag(e, cu, 0);
    code_pred_mode(e, cu, 0);
    code_part_size(e, cu, 0, cu->depth);
    encode_pred_info(e, cu, 0);
    encode_coeff(e, cu, 0);
    *bits += written_bits(e);
  }
}

static void yuv_subtract(yuv_t *dst, const yuv_t *a, const yuv_t *b, int w) {
  for (int c = 0; c < 3; c++) {
    const int n = c ? w >> 1 : w, s = ystride(c);
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++) dst->c[c][y * s + x] = (int16_t)(a->c[c][y * s + x] - b->c[c][y * s + x]);
  }
}
static void yuv_add_clip(yuv_t *dst, const yuv_t *p, const yuv_t *r, int w) {
  for (int c = 0; c < 3; c++) {
    const int n = c ? w >> 1 : w, s = ystride(c);
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++) {
        const int v = p->c[c][y * s + x] + r->c[c][y * s + x];
        dst->c[c][y * s + x] = (int16_t)(v < 0 ? 0 : v > 255 ? 255 : v);
      }
  }
}
static void yuv_copy(yuv_t *dst, const yuv_t *src, int w) {
  for (int c = 0; c < 3; c++) {
    const int n = c ? w >> 1 : w, s = ystride(c);
    for (int y = 0; y < n; y++) memcpy(&dst->c[c][y * s], &src->c[c][y * s], sizeof(int16_t) * n);
  }
}
static void yuv_clear(yuv_t *dst, int w) {
  for (int c = 0; c < 3; c++) {
    const int n = c ? w >> 1 : w, s = ystride(c);
    for (int y = 0; y < n; y++) memset(&dst->c[c][y * s], 0, sizeof(int16_t) * n);
  }
}
static uint32_t yuv_dist(const hm_enc *e, yuv_t *a, yuv_t *b, int w) {
  uint32_t d = 0;
  for (int c = 0; c < 3; c++) {
    const int n = c ? w >> 1 : w;
    d += dist_part(e, a->c[c], ystride(c), b->c[c], ystride(c), n, n, c);
  }
  return d;
}

static void enc_res_rd_inter(hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *pred, yuv_t *resi, yuv_t *resi_best, yuv_t *reco,
                             int skip_residual) {
  const int W = cu->width, depth = cu->depth;
  if (skip_residual) {
    cu_set_all(cu, F_SKIP, 1);
    yuv_clear(resi, W);
    yuv_copy(reco, pred, W);
    const uint32_t dist = yuv_dist(e, reco, org, W);
    e->cur = &e->goon;
    load(e->cur, &e->rd[depth][CI_CURR_BEST]);
    reset_bits(e);
    code_skip_flag(e, cu, 0);
    code_merge_index(e, cu, 0);
    const uint32_t bits = written_bits(e);
    cu->bits = bits; cu->dist = dist;
    cu_measure_ssim(e, cu, org, reco);
    cu->cost = cu_cost(e, cu, bits, dist);
    load(&e->rd[depth][CI_TEMP_BEST], e->cur);
    return;
  }
  yuv_subtract(resi, org, pred, W);
  tu_t t0;
  tu_root(&t0, cu, 0);
  double nz_cost = 0;
  uint32_t nz_bits = 0, nz_dist = 0, z_dist = 0;
  e->cur = &e->goon;
  load(e->cur, &e->rd[depth][CI_CURR_BEST]);
  estimate_inter_residual_qt(e, cu, resi, &nz_cost, &nz_bits, &nz_dist, &z_dist, &t0);
  reset_bits(e);
  cbin(e, X_ROOT_CBF, 0); /* encodeQtRootCbfZero */
  const uint32_t zero_bits = written_bits(e);
  const double zero_cost = rd_cost(e, zero_bits, z_dist);
  if (zero_cost < nz_cost || !cu_qt_root_cbf(cu, 0)) {
    for (int i = 0; i < cu->nparts; i++) {
      cu->p[i].tr_idx = 0;
      cu->p[i].cbf[0] = cu->p[i].cbf[1] = cu->p[i].cbf[2] = 0;
      cu->p[i].ts[0] = cu->p[i].ts[1] = cu->p[i].ts[2] = 0;
    }
  } else set_inter_residual_qt_data(e, cu, NULL, 0, &t0);
  load(e->cur, &e->rd[depth][CI_CURR_BEST]);
  uint32_t final_bits = 0;
  add_symbol_bits_inter(e, cu, &final_bits);
  if (!cu_qt_root_cbf(cu, 0)) yuv_clear(resi_best, W);
  else set_inter_residual_qt_data(e, cu, resi_best, 1, &t0);
  load(&e->rd[depth][CI_TEMP_BEST], e->cur);
  yuv_add_clip(reco, pred, resi_best, W);
  const uint32_t final_dist = yuv_dist(e, reco, org, W);
  cu->bits = final_bits; cu->dist = final_dist;
  cu_measure_ssim(e, cu, org, reco);
  cu->cost = cu_cost(e, cu, final_bits, final_dist);
}

/* ============================================================================================
 * predInterSearch (TEncSearch.cpp:2912), P slices: AMVP (xEstimateMvPredAMVP :3413 with
 * xGetTemplateCost :3619), xMotionEstimation (:3663), xCheckBestMVP (:3567), merge estimation
 * for non-2Nx2N PUs (xMergeEstimation :2832) and AMP_MRG (:3004).
 * ========================================================================================== */
static uint32_t satd_luma_pu(hm_enc *e, yuv_t *org, yuv_t *pred, int rx, int ry, int w, int h) {
  (void)e;
  return hvxo_satd(yaddr(org, 0, rx, ry), 64, yaddr(pred, 0, rx, ry), 64, w, h);
}
static uint32_t template_cost(hm_enc *e, const hm_cu *cu, int ps, int pu, yuv_t *org, int list, int ref_idx, const int16_t *mvc,
                              int mvp_idx) {
  const hvxo_hm_pic *P = e->pic;
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, &a, &w, &h);
  part_position(cu, ps, pu, &xp, &yp, &w, &h);
  /* xPredInterBlk (luma, uni, 8-bit output) at the clipped candidate */
  hvx_mc_job j;
  memset(&j, 0, sizeof(j));
  j.pic_w = P->w; j.pic_h = P->h; j.max_cu = 64;
  j.cu_x = cu->x; j.cu_y = cu->y;
  j.pu_x = xp; j.pu_y = yp; j.w = w; j.h = h;
  j.ref[0] = P->ref_plane_idx[list][ref_idx];
  j.ref[1] = -1;
  j.mv_x[0] = mvc[0]; j.mv_y[0] = mvc[1];
  static _Thread_local int16_t out[64 * 64 + 2 * 32 * 32];
  hvxo_mc(P->ref_planes16, P->ref_stride16[0], P->ref_stride16[1], &j, out);
  const uint32_t sad = hvxo_sad(out, w, yaddr(org, 0, xp - cu->x, yp - cu->y), 64, w, h, 0);
  (void)mvp_idx;
  return (uint32_t)rd_cost_sad(e, 1 /* m_auiMVPIdxCost[idx][2] */, sad);
}
/* xEstimateMvPredAMVP (:3413); *dist_bip (puiDistBiP) takes the best template cost */
static void est_mvp_amvp(hm_enc *e, hm_cu *cu, int ps, int pu, yuv_t *org, int list, int ref_idx, amvp_t *in, int16_t *pred,
                         int *mvp_idx, int *mvp_num, uint32_t *dist_bip) {
  fill_mvp_cand(e, cu, ps, pu, list, ref_idx, in);
  int best = 0;
  if (in->n <= 1) {
    pred[0] = in->c[0][0]; pred[1] = in->c[0][1]; *mvp_idx = 0; *mvp_num = in->n;
    if (e->pic->mvd_l1_zero && list == 1) *dist_bip = template_cost(e, cu, ps, pu, org, list, ref_idx, pred, 0);
    return;
  }
  uint32_t best_cost = MAXU32;
  for (int i = 0; i < in->n; i++) {
    const uint32_t c = template_cost(e, cu, ps, pu, org, list, ref_idx, in->c[i], i);
    if (best_cost > c) { best_cost = c; best = i; *dist_bip = c; }
  }
  pred[0] = in->c[best][0]; pred[1] = in->c[best][1];
  *mvp_idx = best;
  *mvp_num = in->n;
}
static uint32_t eg_bits(int v) { return hvxo_eg_bits(v); }
static void check_best_mvp(hm_enc *e, const amvp_t *in, const int16_t *mv, int16_t *pred, int *mvp_idx, uint32_t *bits,
                           uint32_t *cost) {
  if (in->n < 2) return;
  int best = *mvp_idx;
  const int org_bits = (int)(eg_bits(mv[0] - pred[0]) + eg_bits(mv[1] - pred[1])) + 1;
  int best_bits = org_bits;
  for (int i = 0; i < in->n; i++) {
    if (i == *mvp_idx) continue;
    const int b = (int)(eg_bits(mv[0] - in->c[i][0]) + eg_bits(mv[1] - in->c[i][1])) + 1;
    if (b < best_bits) { best_bits = b; best = i; }
  }
  if (best != *mvp_idx) {
    pred[0] = in->c[best][0]; pred[1] = in->c[best][1];
    *mvp_idx = best;
    const uint32_t ob = *bits;
    *bits = ob - (uint32_t)org_bits + (uint32_t)best_bits;
    *cost = (*cost - mv_cost_bits(e, ob)) + mv_cost_bits(e, *bits);
  }
}
/* xMotionEstimation (uni) through the pinned oracle ME */
static void motion_estimation(hm_enc *e, hm_cu *cu, int ps, int pu, int list, int ref_idx, const int16_t *pred, int16_t *mv,
                              uint32_t *bits, uint32_t *cost) {
  const hvxo_hm_pic *P = e->pic;
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, &a, &w, &h);
  part_position(cu, ps, pu, &xp, &yp, &w, &h);
  hvx_me_job j;
  memset(&j, 0, sizeof(j));
  j.pic_w = P->w; j.pic_h = P->h; j.max_cu = 64;
  j.cu_x = cu->x; j.cu_y = cu->y;
  j.pu_x = xp; j.pu_y = yp; j.w = w; j.h = h;
  j.pred_x = pred[0]; j.pred_y = pred[1];
  j.use_int2nx2n = (ps != SIZE_2Nx2N || cu->depth != 0);
  j.i2_x = e->int2n[list][ref_idx][0];
  j.i2_y = e->int2n[list][ref_idx][1];
  j.bits_in = (int32_t)*bits;
  j.search_range = P->search_range;
  j.lambda_motion = P->lambda_motion;
  j.flags = HVX_ME_FEN | HVX_ME_HADME | HVX_ME_SMOOTHMV;
  hvx_me_result r;
  const int pi = P->ref_plane_idx[list][ref_idx];
  hvxo_motion_estimation(P->org8, P->org8_stride, P->ref_planes8[pi], P->ref_stride8, &j, &r);
  if (ps == SIZE_2Nx2N) { e->int2n[list][ref_idx][0] = (int16_t)r.mv_int_x; e->int2n[list][ref_idx][1] = (int16_t)r.mv_int_y; }
  mv[0] = (int16_t)r.mv_x; mv[1] = (int16_t)r.mv_y;
  *bits = r.bits;
  *cost = r.cost;
}
/* xMergeEstimation (:2832) */
static void merge_estimation(hm_enc *e, hm_cu *cu, int ps, int pu, yuv_t *org, int *inter_dir, mvfield_t *mf, int *merge_idx,
                             uint32_t *cost) {
  mvfield_t f[10];
  int dirs[5];
  int a, w, h;
  part_index_size(cu, ps, pu, &a, &w, &h);
  /* Log2ParallelMergeLevel 2: getInterMergeCandidates of this PU */
  const int n = merge_candidates(e, cu, ps, pu, f, dirs);
  if (cu->width == 8 && (w < 8 || h < 8)) /* xRestrictBipredMergeCand (isBipredRestriction) */
    for (int i = 0; i < n; i++)
      if (dirs[i] == 3) { dirs[i] = 1; f[2 * i + 1].mv[0] = f[2 * i + 1].mv[1] = 0; f[2 * i + 1].ref = -1; }
  *cost = MAXU32;
  int xp, yp;
  part_position(cu, ps, pu, &xp, &yp, &w, &h);
  for (int i = 0; i < n; i++) {
    pu_set_mvfield(cu, ps, pu, 0, f[2 * i].mv[0], f[2 * i].mv[1], f[2 * i].ref);
    pu_set_mvfield(cu, ps, pu, 1, f[2 * i + 1].mv[0], f[2 * i + 1].mv[1], f[2 * i + 1].ref);
    /* xGetInterPredictionError (:2809): MC of REF_PIC_LIST_X from the CU's fields, luma Hadamard */
    mc_pu(e, cu, ps, pu, -1, &e->tmp_yuv_pred);
    uint32_t c = satd_luma_pu(e, org, &e->tmp_yuv_pred, xp - cu->x, yp - cu->y, w, h);
    uint32_t b = (uint32_t)i + 1;
    if (i == e->pic->max_merge - 1) b--;
    c += mv_cost_bits(e, b);
    if (c < *cost) {
      *cost = c;
      mf[0] = f[2 * i];
      mf[1] = f[2 * i + 1];
      *inter_dir = dirs[i];
      *merge_idx = i;
    }
  }
}
/* xMotionEstimation with bBi (TEncSearch.cpp:3663, :3686-3696, :3710-3712, :3726-3729): the target
 * is m_cYuvPredTemp = 2 * org - m_acYuvPred[other list] (TComYuv::removeHighFreq, TComYuv.cpp:409,
 * no clipping: ClipForBiPredMEEnabled is off), the full search of +-BipredSearchRange around the
 * list's current MV (rcMv on entry), the final cost weighted by 0.5 */
static void motion_estimation_bi(hm_enc *e, hm_cu *cu, int ps, int pu, yuv_t *org, int list, int ref_idx, const int16_t *pred,
                                 int16_t *mv, uint32_t *bits, uint32_t *cost) {
  const hvxo_hm_pic *P = e->pic;
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, &a, &w, &h);
  part_position(cu, ps, pu, &xp, &yp, &w, &h);
  const int rx = xp - cu->x, ry = yp - cu->y;
  yuv_t *tg = &e->yuv_pred_tmp;
  const yuv_t *other = &e->yuv_pred_l[1 - list];
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const int o = (ry + y) * 64 + rx + x;
      tg->c[0][o] = (int16_t)(2 * org->c[0][o] - other->c[0][o]);
    }
  hvx_me_job j;
  memset(&j, 0, sizeof(j));
  j.pic_w = P->w; j.pic_h = P->h; j.max_cu = 64;
  j.cu_x = cu->x; j.cu_y = cu->y;
  j.pu_x = xp; j.pu_y = yp; j.w = w; j.h = h;
  j.pred_x = pred[0]; j.pred_y = pred[1];
  j.center_x = mv[0]; j.center_y = mv[1];
  j.bits_in = (int32_t)*bits;
  j.search_range = P->bipred_range;
  j.lambda_motion = P->lambda_motion;
  j.flags = HVX_ME_FEN | HVX_ME_HADME | HVX_ME_BI;
  hvx_me_result r;
  const int pi = P->ref_plane_idx[list][ref_idx];
  hvxo_me_full_pat(tg->c[0] + ry * 64 + rx, 64, P->ref_planes8[pi], P->ref_stride8, &j, &r);
  mv[0] = (int16_t)r.mv_x; mv[1] = (int16_t)r.mv_y;
  *bits = r.bits;
  *cost = r.cost;
}
/* xGetBlkBits (:3509) */
static void blk_bits(int ps, int is_p, int pu, int last_mode, uint32_t *b) {
  static const uint32_t hor[2][3][3] = {{{0, 0, 3}, {0, 0, 0}, {0, 0, 0}}, {{5, 7, 7}, {7, 5, 7}, {6, 6, 6}}};
  static const uint32_t ver[2][3][3] = {{{0, 2, 3}, {0, 0, 0}, {0, 0, 0}}, {{5, 7, 7}, {5, 5, 7}, {6, 6, 6}}};
  if (ps == SIZE_2Nx2N || ps == SIZE_NxN) { b[0] = is_p ? 1 : 3; b[1] = 3; b[2] = 5; return; }
  if (is_p) { b[0] = 3; b[1] = 0; b[2] = 0; return; }
  const uint32_t *t = (ps == SIZE_2NxN || ps == SIZE_2NxnU || ps == SIZE_2NxnD) ? hor[pu][last_mode] : ver[pu][last_mode];
  b[0] = t[0]; b[1] = t[1]; b[2] = t[2];
}
/* the reference index bits of predInterSearch (:3021-3028) */
static uint32_t ref_bits(int r, int n) {
  if (n <= 1) return 0;
  return (uint32_t)r + 1 - (r == n - 1 ? 1u : 0u);
}
/* predInterSearch (:2912), P and B slices */
static int pred_inter_search(hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *pred, int use_mrg) {
  const hvxo_hm_pic *P = e->pic;
  const int ps = cu->p[0].part, npart = num_parts_of(ps);
  const int isb = P->slice_type == B_SLICE, ndir = isb ? 2 : 1;
  int last_mode = 0;
  /* declared outside the PU loop in the reference (:2937-2969): kept across PUs */
  int16_t mv[2][2] = {{0, 0}, {0, 0}};
  int ref[2] = {0, 0};
  int16_t mvtemp[2][4][2], mvpred[2][4][2], mvpredbi[2][4][2];
  int mvp_idx[2][4], mvp_num[2][4], mvp_idx_bi[2][4];
  amvp_t amvp[2][4];
  int best_bip_ref_l1 = 0, best_bip_mvp_l1 = 0;
  uint32_t bip_dist_temp = MAXU32;
  memset(mvtemp, 0, sizeof(mvtemp));
  memset(mvpred, 0, sizeof(mvpred));
  for (int pu = 0; pu < npart; pu++) {
    uint32_t cost[2] = {MAXU32, MAXU32}, cost_bi = MAXU32, bits[3] = {0, 0, 0};
    uint32_t best_bip_dist = MAXU32;
    uint32_t cost_l0[4] = {MAXU32, MAXU32, MAXU32, MAXU32}, bits_l0[4] = {0, 0, 0, 0};
    int16_t mv_valid_l1[2] = {0, 0};
    int ref_valid_l1 = 0;
    uint32_t bits_valid_l1 = MAXU32, cost_valid_l1 = MAXU32;
    int16_t mvbi[2][2] = {{0, 0}, {0, 0}};
    int refbi[2] = {0, 0};
    uint32_t mb[3];
    blk_bits(ps, !isb, pu, last_mode, mb);
    int a, w, h;
    part_index_size(cu, ps, pu, &a, &w, &h);
    const int test_normal = !(use_mrg && cu->width > 8 && npart == 2);
    if (test_normal) {
      /* uni-directional prediction (:3014-3093) */
      for (int l = 0; l < ndir; l++) {
        for (int r = 0; r < P->nref[l]; r++) {
          uint32_t bt = mb[l] + ref_bits(r, P->nref[l]), ct;
          uint32_t dist_bip = bip_dist_temp;
          est_mvp_amvp(e, cu, ps, pu, org, l, r, &amvp[l][r], mvpred[l][r], &mvp_idx[l][r], &mvp_num[l][r], &dist_bip);
          bip_dist_temp = dist_bip;
          pu_set(cu, ps, pu, PU_MVP_IDX, l, mvp_idx[l][r]);
          pu_set(cu, ps, pu, PU_MVP_NUM, l, mvp_num[l][r]);
          if (P->mvd_l1_zero && l == 1 && bip_dist_temp < best_bip_dist) {
            best_bip_dist = bip_dist_temp;
            best_bip_mvp_l1 = mvp_idx[l][r];
            best_bip_ref_l1 = r;
          }
          bt += 1; /* m_auiMVPIdxCost[idx][AMVP_MAX_NUM_CANDS] */
          if (l == 1 && P->l1_to_l0[r] >= 0) {
            /* FastMEForGenBLowDelayEnabled (:3042-3055): the L0 search of the same picture, re-costed */
            const int m = P->l1_to_l0[r];
            mvtemp[1][r][0] = mvtemp[0][m][0]; mvtemp[1][r][1] = mvtemp[0][m][1];
            ct = cost_l0[m];
            ct -= mv_cost_bits(e, bits_l0[m]);
            bt += eg_bits(mvtemp[1][r][0] - mvpred[1][r][0]) + eg_bits(mvtemp[1][r][1] - mvpred[1][r][1]);
            ct += mv_cost_bits(e, bt);
          } else {
            motion_estimation(e, cu, ps, pu, l, r, mvpred[l][r], mvtemp[l][r], &bt, &ct);
          }
          check_best_mvp(e, &amvp[l][r], mvtemp[l][r], mvpred[l][r], &mvp_idx[l][r], &bt, &ct);
          if (l == 0) { cost_l0[r] = ct; bits_l0[r] = bt; }
          if (ct < cost[l]) { cost[l] = ct; bits[l] = bt; mv[l][0] = mvtemp[l][r][0]; mv[l][1] = mvtemp[l][r][1]; ref[l] = r; }
          if (l == 1 && ct < cost_valid_l1 && P->l1_to_l0[r] < 0) {
            cost_valid_l1 = ct; bits_valid_l1 = bt;
            mv_valid_l1[0] = mvtemp[l][r][0]; mv_valid_l1[1] = mvtemp[l][r][1];
            ref_valid_l1 = r;
          }
        }
      }
      /* bi-directional prediction (:3096-3251), FEN: one iteration */
      if (isb && !(cu->width == 8 && (w < 8 || h < 8))) { /* isBipredRestriction (TComDataCU.cpp:2773) */
        mvbi[0][0] = mv[0][0]; mvbi[0][1] = mv[0][1]; mvbi[1][0] = mv[1][0]; mvbi[1][1] = mv[1][1];
        refbi[0] = ref[0]; refbi[1] = ref[1];
        memcpy(mvpredbi, mvpred, sizeof(mvpred));
        memcpy(mvp_idx_bi, mvp_idx, sizeof(mvp_idx));
        uint32_t motbits[2];
        if (P->mvd_l1_zero) {
          const int br = best_bip_ref_l1;
          pu_set(cu, ps, pu, PU_MVP_IDX, 1, best_bip_mvp_l1);
          mvp_idx_bi[1][br] = best_bip_mvp_l1;
          mvpredbi[1][br][0] = amvp[1][br].c[best_bip_mvp_l1][0];
          mvpredbi[1][br][1] = amvp[1][br].c[best_bip_mvp_l1][1];
          mvbi[1][0] = mvpredbi[1][br][0]; mvbi[1][1] = mvpredbi[1][br][1];
          refbi[1] = br;
          pu_set_mvfield(cu, ps, pu, 1, mvbi[1][0], mvbi[1][1], br);
          mc_pu(e, cu, ps, pu, 1, &e->yuv_pred_l[1]);
          motbits[0] = bits[0] - mb[0];
          motbits[1] = mb[1] + ref_bits(br, P->nref[1]) + 1;
          bits[2] = mb[2] + motbits[0] + motbits[1];
          mvtemp[1][br][0] = mvbi[1][0]; mvtemp[1][br][1] = mvbi[1][1];
        } else {
          motbits[0] = bits[0] - mb[0];
          motbits[1] = bits[1] - mb[1];
          bits[2] = mb[2] + motbits[0] + motbits[1];
        }
        /* UseFastEnc: iNumIter 1, the list searched is the costlier uni list */
        int l = cost[0] <= cost[1] ? 1 : 0;
        if (!P->mvd_l1_zero) {
          pu_set_mv(cu, ps, pu, 1 - l, mv[1 - l][0], mv[1 - l][1]);
          pu_set_ref(cu, ps, pu, 1 - l, ref[1 - l]);
          mc_pu(e, cu, ps, pu, 1 - l, &e->yuv_pred_l[1 - l]);
        } else l = 0;
        int changed = 0;
        for (int r = 0; r < P->nref[l]; r++) {
          uint32_t bt = mb[2] + motbits[1 - l] + ref_bits(r, P->nref[l]) + 1, ct;
          motion_estimation_bi(e, cu, ps, pu, org, l, r, mvpredbi[l][r], mvtemp[l][r], &bt, &ct);
          check_best_mvp(e, &amvp[l][r], mvtemp[l][r], mvpredbi[l][r], &mvp_idx_bi[l][r], &bt, &ct);
          if (ct < cost_bi) {
            changed = 1;
            mvbi[l][0] = mvtemp[l][r][0]; mvbi[l][1] = mvtemp[l][r][1];
            refbi[l] = r;
            cost_bi = ct;
            motbits[l] = bt - mb[2] - motbits[1 - l];
            bits[2] = bt;
          }
        }
        if (!changed && cost_bi <= cost[0] && cost_bi <= cost[1]) {
          check_best_mvp(e, &amvp[0][refbi[0]], mvbi[0], mvpredbi[0][refbi[0]], &mvp_idx_bi[0][refbi[0]], &bits[2], &cost_bi);
          if (!P->mvd_l1_zero)
            check_best_mvp(e, &amvp[1][refbi[1]], mvbi[1], mvpredbi[1][refbi[1]], &mvp_idx_bi[1][refbi[1]], &bits[2], &cost_bi);
        }
      }
    }
    /* clear the PU's motion (:3257-3265) */
    pu_set_mvfield(cu, ps, pu, 0, 0, 0, -1);
    pu_set_mvfield(cu, ps, pu, 1, 0, 0, -1);
    pu_set_mvd(cu, ps, pu, 0, 0, 0);
    pu_set_mvd(cu, ps, pu, 1, 0, 0);
    pu_set(cu, ps, pu, PU_MVP_IDX, 0, -1); pu_set(cu, ps, pu, PU_MVP_NUM, 0, -1);
    pu_set(cu, ps, pu, PU_MVP_IDX, 1, -1); pu_set(cu, ps, pu, PU_MVP_NUM, 1, -1);
    uint32_t me_bits = 0;
    /* list 1 only through a picture list 0 does not hold (:3269-3272) */
    mv[1][0] = mv_valid_l1[0]; mv[1][1] = mv_valid_l1[1];
    ref[1] = ref_valid_l1;
    bits[1] = bits_valid_l1;
    cost[1] = cost_valid_l1;
    if (test_normal) {
      if (cost_bi <= cost[0] && cost_bi <= cost[1]) {
        last_mode = 2;
        pu_set_mv(cu, ps, pu, 0, mvbi[0][0], mvbi[0][1]);
        pu_set_ref(cu, ps, pu, 0, refbi[0]);
        pu_set_mv(cu, ps, pu, 1, mvbi[1][0], mvbi[1][1]);
        pu_set_ref(cu, ps, pu, 1, refbi[1]);
        pu_set_mvd(cu, ps, pu, 0, mvbi[0][0] - mvpredbi[0][refbi[0]][0], mvbi[0][1] - mvpredbi[0][refbi[0]][1]);
        pu_set_mvd(cu, ps, pu, 1, mvbi[1][0] - mvpredbi[1][refbi[1]][0], mvbi[1][1] - mvpredbi[1][refbi[1]][1]);
        pu_set(cu, ps, pu, PU_INTER_DIR, 0, 3);
        pu_set(cu, ps, pu, PU_MVP_IDX, 0, mvp_idx_bi[0][refbi[0]]);
        pu_set(cu, ps, pu, PU_MVP_NUM, 0, mvp_num[0][refbi[0]]);
        pu_set(cu, ps, pu, PU_MVP_IDX, 1, mvp_idx_bi[1][refbi[1]]);
        pu_set(cu, ps, pu, PU_MVP_NUM, 1, mvp_num[1][refbi[1]]);
        me_bits = bits[2];
      } else if (cost[0] <= cost[1]) {
        last_mode = 0;
        pu_set_mv(cu, ps, pu, 0, mv[0][0], mv[0][1]);
        pu_set_ref(cu, ps, pu, 0, ref[0]);
        pu_set_mvd(cu, ps, pu, 0, mv[0][0] - mvpred[0][ref[0]][0], mv[0][1] - mvpred[0][ref[0]][1]);
        pu_set(cu, ps, pu, PU_INTER_DIR, 0, 1);
        pu_set(cu, ps, pu, PU_MVP_IDX, 0, mvp_idx[0][ref[0]]);
        pu_set(cu, ps, pu, PU_MVP_NUM, 0, mvp_num[0][ref[0]]);
        me_bits = bits[0];
      } else {
        last_mode = 1;
        pu_set_mv(cu, ps, pu, 1, mv[1][0], mv[1][1]);
        pu_set_ref(cu, ps, pu, 1, ref[1]);
        pu_set_mvd(cu, ps, pu, 1, mv[1][0] - mvpred[1][ref[1]][0], mv[1][1] - mvpred[1][ref[1]][1]);
        pu_set(cu, ps, pu, PU_INTER_DIR, 0, 2);
        pu_set(cu, ps, pu, PU_MVP_IDX, 1, mvp_idx[1][ref[1]]);
        pu_set(cu, ps, pu, PU_MVP_NUM, 1, mvp_num[1][ref[1]]);
        me_bits = bits[1];
      }
    }
    if (ps != SIZE_2Nx2N) {
      uint32_t me_cost = MAXU32;
      int xp, yp;
      part_position(cu, ps, pu, &xp, &yp, &w, &h);
      if (test_normal) {
        mc_pu(e, cu, ps, pu, -1, &e->tmp_yuv_pred);
        const uint32_t err = satd_luma_pu(e, org, &e->tmp_yuv_pred, xp - cu->x, yp - cu->y, w, h);
        me_cost = err + mv_cost_bits(e, me_bits);
      }
      const hm_part save = cu->p[a];
      int mrg_dir = 0, mrg_idx = 0;
      mvfield_t mrg[2] = {{{0, 0}, -1}, {{0, 0}, -1}};
      uint32_t mrg_cost = MAXU32;
      merge_estimation(e, cu, ps, pu, org, &mrg_dir, mrg, &mrg_idx, &mrg_cost);
      if (mrg_cost < me_cost) {
        pu_set(cu, ps, pu, PU_MERGE, 0, 1);
        pu_set(cu, ps, pu, PU_MERGE_IDX, 0, mrg_idx);
        pu_set(cu, ps, pu, PU_INTER_DIR, 0, mrg_dir);
        pu_set_mvfield(cu, ps, pu, 0, mrg[0].mv[0], mrg[0].mv[1], mrg[0].ref);
        pu_set_mvfield(cu, ps, pu, 1, mrg[1].mv[0], mrg[1].mv[1], mrg[1].ref);
        pu_set_mvd(cu, ps, pu, 0, 0, 0);
        pu_set_mvd(cu, ps, pu, 1, 0, 0);
        pu_set(cu, ps, pu, PU_MVP_IDX, 0, -1); pu_set(cu, ps, pu, PU_MVP_NUM, 0, -1);
        pu_set(cu, ps, pu, PU_MVP_IDX, 1, -1); pu_set(cu, ps, pu, PU_MVP_NUM, 1, -1);
      } else {
        pu_set(cu, ps, pu, PU_MERGE, 0, 0);
        pu_set(cu, ps, pu, PU_INTER_DIR, 0, save.inter_dir);
        pu_set_mvfield(cu, ps, pu, 0, save.mv[0][0], save.mv[0][1], save.ref[0]);
        pu_set_mvfield(cu, ps, pu, 1, save.mv[1][0], save.mv[1][1], save.ref[1]);
      }
    }
    mc_pu(e, cu, ps, pu, -1, pred);
  }
  return 1;
}

/* ============================================================================================
 * Intra: estIntraPredLumaQT (TEncSearch.cpp:2176), xRecurIntraCodingLumaQT (:1390),
 * xIntraCodingTUBlock (:1088), estIntraPredChromaQT (:2563), xRecurIntraChromaCodingQT (:1913),
 * xGetIntraBitsQT (:1051), xEncIntraHeader (:976), xEncSubdivCbfQT (:866), xEncCoeffQT (:936),
 * with initIntraPatternChType (TComPattern.cpp:115) on the picture reconstruction.
 * ========================================================================================== */
/* the reference samples of a TU: availability per 4x4 partition (isAboveLeftAvailable etc.,
 * TComPattern.cpp:570-760) and the reconstruction at the border positions */
static void intra_border(hm_enc *e, const hm_cu *cu, const tu_t *t, int comp, int16_t *raw, uint32_t *avail, int *unit_log2) {
  const int c = comp, s = c ? 1 : 0;
  const int w = t->w[c], h = t->h[c];
  const int unit = c ? 2 : 4;
  const int wu = w / unit, hu = h / unit;
  const int rel = tu_abs_rel(t);
  const int lt = cu->zidx + rel;
  const int rt = R2Z[Z2R[lt] + wu - 1], lb = R2Z[Z2R[lt] + (hu - 1) * 16];
  const int lunits = hu * 2;
  avail[0] = avail[1] = avail[2] = 0;
#define SETA(i, v) do { if (v) avail[(i) >> 5] |= 1u << ((i) & 31); } while (0)
  SETA(lunits, get_pu_above_left(e, cu, lt).valid);
  for (int k = 0; k < wu; k++) SETA(lunits + 1 + k, get_pu_above(e, cu, R2Z[Z2R[lt] + k], 0).valid);
  for (int k = 1; k <= wu; k++) SETA(lunits + wu + k, get_pu_above_right(e, cu, rt, k).valid);
  for (int k = 0; k < hu; k++) SETA(lunits - 1 - k, get_pu_left(e, cu, R2Z[Z2R[lt] + k * 16]).valid);
  for (int k = 1; k <= hu; k++) SETA(hu - k, get_pu_below_left(e, cu, lb, k).valid);
#undef SETA
  *unit_log2 = c ? 1 : 2;
  /* raw samples: B layout of hvxo_intra_fill (above-left, above row 2w, left column 2h) */
  const int x0 = (cu->x >> s) + t->x0[c], y0 = (cu->y >> s) + t->y0[c];
  const int W = (e->pic->w >> s), H = (e->pic->h >> s);
  const int n = w;
  for (int k = 0; k <= 4 * n; k++) raw[k] = 0;
  /* reads stay inside the whole-CTU reconstruction buffer (unavailable units are substituted by
     hvxo_intra_fill, so what is read there does not matter) */
  const int RW = (((e->pic->w + 63) >> 6) << 6) >> s, RH = (((e->pic->h + 63) >> 6) << 6) >> s;
  (void)W; (void)H;
#define REC(x, y) (((x) >= 0 && (y) >= 0 && (x) < RW && (y) < RH) ? *rec_at(e, c, (x), (y)) : 0)
  raw[0] = REC(x0 - 1, y0 - 1);
  for (int k = 0; k < 2 * n; k++) raw[1 + k] = REC(x0 + k, y0 - 1);
  for (int k = 0; k < 2 * n; k++) raw[2 * n + 1 + k] = REC(x0 - 1, y0 + k);
#undef REC
}
/* predIntraAng for a TU of the CU into pred (stride ystride(comp)) */
static void intra_predict_tu(hm_enc *e, const hm_cu *cu, const tu_t *t, int comp, int mode, int16_t *pred) {
  const int n = t->w[comp];
  int16_t raw[4 * 64 + 1], B[4 * 64 + 1], F[4 * 64 + 1];
  uint32_t avail[3];
  int ul;
  intra_border(e, cu, t, comp, raw, avail, &ul);
  hvxo_intra_fill(raw, avail, n, ul, B);
  const int16_t *src = B;
  if (comp == 0 && hvxo_intra_use_filter(mode, n, 1)) {
    hvxo_intra_filter(B, n, 1, 1, F);
    src = F;
  }
  uint8_t p8[64 * 64];
  hvxo_intra_pred(src, n, comp == 0, mode, p8);
  for (int y = 0; y < n; y++)
    for (int x = 0; x < n; x++) pred[y * ystride(comp) + x] = p8[y * n + x];
}

static uint32_t intra_bits_qt(hm_enc *e, hm_cu *cu, const tu_t *t, int luma, int chroma);

/* xIntraCodingTUBlock (:1088) */
static void intra_coding_tu(hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *pred, yuv_t *resi, uint32_t *dist, int comp, const tu_t *t,
                            int save_load) {
  if (!tu_proc(t, comp)) return;
  const int rel = tu_abs_rel(t);
  const int w = t->w[comp], h = t->h[comp], x0 = t->x0[comp], y0 = t->y0[comp];
  const int s = ystride(comp);
  int16_t *po = yaddr(org, comp, x0, y0), *pp = yaddr(pred, comp, x0, y0), *pr = yaddr(resi, comp, x0, y0);
  const int layer = qt_layer(t->log2);
  int16_t *prq = yaddr(&e->qt_yuv[layer], comp, x0, y0);
  int32_t *coef = e->qt_coef[comp][layer] + t->off[comp];
  int mode = cu->p[rel].idir[comp ? 1 : 0];
  if (comp && mode == DM_CHROMA_IDX) mode = cu->p[rel].idir[0];
  if (save_load != 2) {
    intra_predict_tu(e, cu, t, comp, mode, pp);
    if (save_load == 1)
      for (int y = 0; y < h; y++) memcpy(&e->shared_pred[comp][y * w], pp + y * s, sizeof(int16_t) * w);
  } else {
    for (int y = 0; y < h; y++) memcpy(pp + y * s, &e->shared_pred[comp][y * w], sizeof(int16_t) * w);
  }
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) pr[y * s + x] = (int16_t)(po[y * s + x] - pp[y * s + x]);
  const int ts = cu->p[tu_abs_rel_c(t, comp)].ts[comp];
  (void)ts;
  estimate_bit(e, w, h, comp ? 1 : 0); /* RDOQ and RDOQTS are both on */
  int32_t abs_sum = 0;
  if (comp == 0) set_tridx(cu, rel, 256 >> (2 * tu_depth_total(t)), tu_depth_rel(t));
  transform_tu(e, cu, t, comp, pr, s, coef, &abs_sum);
  if (abs_sum > 0) inv_transform_tu(e, cu, t, comp, coef, pr, s);
  else {
    memset(coef, 0, sizeof(int32_t) * w * h);
    for (int y = 0; y < h; y++) memset(pr + y * s, 0, sizeof(int16_t) * w);
  }
  const int px0 = (cu->x >> (comp ? 1 : 0)) + x0, py0 = (cu->y >> (comp ? 1 : 0)) + y0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int v = pp[y * s + x] + pr[y * s + x];
      v = v < 0 ? 0 : v > 255 ? 255 : v;
      pp[y * s + x] = (int16_t)v;        /* piReco = piPred */
      prq[y * s + x] = (int16_t)v;
      *rec_at(e, comp, px0 + x, py0 + y) = (int16_t)v;
    }
  *dist += dist_part(e, pp, s, po, s, w, h, comp);
}
/* xStoreIntraResultQT (:1758) / xLoadIntraResultQT (:1793) */
static void intra_store(hm_enc *e, int comp, const tu_t *t) {
  if (!tu_proc(t, comp)) return;
  const int layer = qt_layer(t->log2), w = t->w[comp], h = t->h[comp];
  memcpy(e->qt_tu_coef[comp], e->qt_coef[comp][layer] + t->off[comp], sizeof(int32_t) * w * h);
  for (int y = 0; y < h; y++)
    memcpy(yaddr(&e->qt_ts_yuv, comp, t->x0[comp], t->y0[comp] + y), yaddr(&e->qt_yuv[layer], comp, t->x0[comp], t->y0[comp] + y),
           sizeof(int16_t) * w);
}
static void intra_load(hm_enc *e, const hm_cu *cu, int comp, const tu_t *t) {
  if (!tu_proc(t, comp)) return;
  const int layer = qt_layer(t->log2), w = t->w[comp], h = t->h[comp], s = comp ? 1 : 0;
  memcpy(e->qt_coef[comp][layer] + t->off[comp], e->qt_tu_coef[comp], sizeof(int32_t) * w * h);
  for (int y = 0; y < h; y++) {
    memcpy(yaddr(&e->qt_yuv[layer], comp, t->x0[comp], t->y0[comp] + y), yaddr(&e->qt_ts_yuv, comp, t->x0[comp], t->y0[comp] + y),
           sizeof(int16_t) * w);
    for (int x = 0; x < w; x++)
      *rec_at(e, comp, (cu->x >> s) + t->x0[comp] + x, (cu->y >> s) + t->y0[comp] + y) =
          *yaddr(&e->qt_yuv[layer], comp, t->x0[comp] + x, t->y0[comp] + y);
  }
}
static void set_cbf_sub(hm_cu *cu, int comp, int rel, int n, int v) { for (int i = 0; i < n; i++) cu->p[rel + i].cbf[comp] = (uint8_t)v; }

static void recur_intra_luma_qt(hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *pred, yuv_t *resi, uint32_t *dist_y, int check_first,
                                double *rd_cost_out, const tu_t *t) {
  const int rel = tu_abs_rel(t), full_depth = tu_depth_total(t), trd = tu_depth_rel(t), l2 = t->log2;
  int check_full = l2 <= 5;
  int check_split = l2 > qt_min_log2(cu, rel);
  /* HHI_RQT_INTRA_SPEEDUP, RDpenalty 0 */
  if (check_first && check_full) check_split = 0;
  double single_cost = MAX_DOUBLE;
  uint32_t single_dist = 0;
  int single_cbf = 0;
  int check_ts = t->w[0] <= 4 && cu->p[rel].part == SIZE_NxN; /* TransformSkipFast */
  int best_mode = 0;
  const int nparts_here = 256 >> (2 * full_depth);
  if (check_full) {
    if (check_ts) {
      load(&e->rd[full_depth][CI_QT_TRAFO_ROOT], e->cur);
      for (int mode = 0; mode < 2; mode++) {
        uint32_t dtmp = 0;
        double ctmp;
        if (tu_proc(t, 0)) {
          set_ts_range(cu, 0, rel, nparts_here, mode);
          intra_coding_tu(e, cu, org, pred, resi, &dtmp, 0, t, mode == 0 ? 1 : 2);
        }
        const int cbf = cbf_at(&cu->p[rel], 0, trd);
        if (mode == 1 && cbf == 0) ctmp = MAX_DOUBLE;
        else {
          const uint32_t b = intra_bits_qt(e, cu, t, 1, 0);
          ctmp = rd_cost(e, b, dtmp);
        }
        if (ctmp < single_cost) {
          single_cost = ctmp;
          single_dist = dtmp;
          single_cbf = cbf;
          best_mode = mode;
          if (best_mode == 0) {
            intra_store(e, 0, t);
            load(&e->rd[full_depth][CI_TEMP_BEST], e->cur);
          }
        }
        if (mode == 0) load(e->cur, &e->rd[full_depth][CI_QT_TRAFO_ROOT]);
      }
      if (tu_proc(t, 0)) set_ts_range(cu, 0, rel, nparts_here, best_mode);
      if (best_mode == 0) {
        intra_load(e, cu, 0, t);
        if (tu_proc(t, 0)) set_cbf_sub(cu, 0, rel, nparts_here, single_cbf << trd);
        load(e->cur, &e->rd[full_depth][CI_TEMP_BEST]);
      }
    } else {
      if (check_split) load(&e->rd[full_depth][CI_QT_TRAFO_ROOT], e->cur);
      single_cost = 0.0;
      if (tu_proc(t, 0)) set_ts_range(cu, 0, rel, nparts_here, 0);
      intra_coding_tu(e, cu, org, pred, resi, &single_dist, 0, t, 0);
      if (check_split) single_cbf = cbf_at(&cu->p[rel], 0, trd);
      const uint32_t b = intra_bits_qt(e, cu, t, 1, 0);
      single_cost = rd_cost(e, b, single_dist);
    }
  }
  if (check_split) {
    if (check_full) {
      load(&e->rd[full_depth][CI_QT_TRAFO_TEST], e->cur);
      load(e->cur, &e->rd[full_depth][CI_QT_TRAFO_ROOT]);
    } else load(&e->rd[full_depth][CI_QT_TRAFO_ROOT], e->cur);
    double split_cost = 0.0;
    uint32_t split_dist = 0;
    int split_cbf = 0;
    tu_t ch;
    tu_child(&ch, t, 0);
    do {
      recur_intra_luma_qt(e, cu, org, pred, resi, &split_dist, check_first, &split_cost, &ch);
      split_cbf |= cbf_at(&cu->p[tu_abs_rel(&ch)], 0, tu_depth_rel(&ch));
    } while (tu_next(&ch, t));
    if (split_cbf)
      for (int i = 0; i < t->step; i++) cu->p[rel + i].cbf[0] |= (uint8_t)(1 << trd);
    load(e->cur, &e->rd[full_depth][CI_QT_TRAFO_ROOT]);
    const uint32_t b = intra_bits_qt(e, cu, t, 1, 0);
    split_cost = rd_cost(e, b, split_dist);
    if (split_cost < single_cost) {
      *dist_y += split_dist;
      *rd_cost_out += split_cost;
      return;
    }
    load(e->cur, &e->rd[full_depth][CI_QT_TRAFO_TEST]);
    set_tridx(cu, rel, nparts_here, trd);
    set_cbf_sub(cu, 0, rel, nparts_here, single_cbf << trd);
    set_ts_range(cu, 0, rel, nparts_here, best_mode);
    /* the single-TU reconstruction back into the picture for the next intra blocks */
    const int layer = qt_layer(l2), w = t->w[0];
    for (int y = 0; y < w; y++)
      for (int x = 0; x < w; x++)
        *rec_at(e, 0, cu->x + t->x0[0] + x, cu->y + t->y0[0] + y) = *yaddr(&e->qt_yuv[layer], 0, t->x0[0] + x, t->y0[0] + y);
  }
  *dist_y += single_dist;
  *rd_cost_out += single_cost;
}
/* xSetIntraResultLumaQT (:1715) */
static void set_intra_result_luma(hm_enc *e, hm_cu *cu, yuv_t *reco, const tu_t *t) {
  const int rel = tu_abs_rel(t);
  if (cu->p[rel].tr_idx == tu_depth_rel(t)) {
    const int layer = qt_layer(t->log2), w = t->w[0];
    if (w) {
      memcpy(cu->coef[0] + t->off[0], e->qt_coef[0][layer] + t->off[0], sizeof(int32_t) * w * w);
      for (int y = 0; y < w; y++)
        memcpy(yaddr(reco, 0, t->x0[0], t->y0[0] + y), yaddr(&e->qt_yuv[layer], 0, t->x0[0], t->y0[0] + y), sizeof(int16_t) * w);
    }
  } else {
    tu_t ch;
    tu_child(&ch, t, 0);
    do set_intra_result_luma(e, cu, reco, &ch); while (tu_next(&ch, t));
  }
}

/* xEncIntraHeader (:976) */
static void enc_intra_header(hm_enc *e, hm_cu *cu, int trd, int rel, int luma, int chroma) {
  if (luma) {
    if (rel == 0) {
      if (e->pic->slice_type != I_SLICE) {
        code_skip_flag(e, cu, 0);
        code_pred_mode(e, cu, 0);
      }
      code_part_size(e, cu, 0, cu->depth);
    }
    if (cu->p[0].part == SIZE_2Nx2N) {
      if (rel == 0) code_intra_dir_luma(e, cu, 0, 0);
    } else {
      const int q = cu->nparts >> 2;
      if (trd > 0 && (rel % q) == 0) code_intra_dir_luma(e, cu, rel, 0);
    }
  }
  if (chroma) {
    if (rel == 0) code_intra_dir_chroma(e, cu, rel); /* 4:2:0: one chroma PU */
  }
}
/* xEncSubdivCbfQT (:866) */
static void enc_subdiv_cbf_qt(hm_enc *e, hm_cu *cu, const tu_t *t, int luma, int chroma) {
  const int rel = tu_abs_rel(t), trd = tu_depth_rel(t);
  const int trmode = cu->p[rel].tr_idx, subdiv = trmode > trd, l2 = t->log2;
  if (cu->p[0].pred == MODE_INTRA && cu->p[0].part == SIZE_NxN && trd == 0) {
  } else if (l2 > 5) {
  } else if (l2 == 2) {
  } else if (l2 == qt_min_log2(cu, rel)) {
  } else if (luma) code_subdiv(e, subdiv, 5 - l2);
  if (chroma)
    for (int c = 1; c < 3; c++)
      if (t->all[c] && (trd == 0 || cbf_at(&cu->p[rel], c, trd - 1))) code_qt_cbf(e, cu, t, c, !subdiv);
  if (subdiv) {
    tu_t ch;
    tu_child(&ch, t, 0);
    do enc_subdiv_cbf_qt(e, cu, &ch, luma, chroma); while (tu_next(&ch, t));
  } else if (luma) code_qt_cbf(e, cu, t, 0, 1);
}
/* xEncCoeffQT (:936) with the QT temp coefficients */
static void enc_coeff_qt(hm_enc *e, hm_cu *cu, const tu_t *t, int comp) {
  const int rel = tu_abs_rel(t), trd = tu_depth_rel(t);
  if (cu->p[rel].tr_idx > trd) {
    tu_t ch;
    tu_child(&ch, t, 0);
    do enc_coeff_qt(e, cu, &ch, comp); while (tu_next(&ch, t));
  } else if (tu_proc(t, comp)) {
    const int crel = tu_abs_rel_c(t, comp);
    if (cbf_at(&cu->p[crel], comp, trd)) /* encodeCoeffNxN checks the cbf at the TU depth */
      code_coeff_nxn(e, cu, t, comp, e->qt_coef[comp][qt_layer(t->log2)] + t->off[comp]);
  }
}
static uint32_t intra_bits_qt(hm_enc *e, hm_cu *cu, const tu_t *t, int luma, int chroma) {
  reset_bits(e);
  enc_intra_header(e, cu, tu_depth_rel(t), tu_abs_rel(t), luma, chroma);
  enc_subdiv_cbf_qt(e, cu, t, luma, chroma);
  if (luma) enc_coeff_qt(e, cu, t, 0);
  if (chroma) { enc_coeff_qt(e, cu, t, 1); enc_coeff_qt(e, cu, t, 2); }
  return written_bits(e);
}

static void est_intra_pred_luma_qt(hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *pred, yuv_t *resi, yuv_t *reco) {
  const hvxo_hm_pic *P = e->pic;
  const int depth = cu->depth;
  const int init_trd = cu->p[0].part == SIZE_2Nx2N ? 0 : 1;
  const int qnp = cu->nparts >> 2;
  uint32_t overall_dist = 0;
  for (int i = 0; i < cu->nparts; i++) cu->p[i].qp = (int8_t)e->slice_qp;
  tu_t tcu, tpu;
  tu_root(&tcu, cu, 0);
  if (init_trd) tu_child(&tpu, &tcu, 0);
  else tpu = tcu;
  do {
    const int poff = tu_abs_rel(&tpu);
    const int n = tpu.w[0];
    /* first pass through the pinned restatement: SATD of 35 modes + xModeBitsIntra + candidate list + MPMs */
    hvx_intra_job j;
    memset(&j, 0, sizeof(j));
    int16_t raw[257];
    int ul;
    intra_border(e, cu, &tpu, 0, raw, j.avail, &ul);
    j.log2_size = log2i(n);
    j.ch_type = 0;
    j.unit_log2 = ul;
    j.flags = HVX_INTRA_STRONG | HVX_INTRA_FAST_MPM;
    {
      nb_t l = get_pu_left(e, cu, cu->zidx + poff), a = get_pu_above(e, cu, cu->zidx + poff, 1);
      j.left_dir = (l.valid && l.p[l.idx].pred == MODE_INTRA) ? l.p[l.idx].idir[0] : 1;
      j.above_dir = (a.valid && a.p[a.idx].pred == MODE_INTRA) ? a.p[a.idx].idir[0] : 1;
    }
    j.ctx_state = e->rd[depth][CI_CURR_BEST].st[X_INTRA];
    j.frac_bits = (int32_t)(e->rd[depth][CI_CURR_BEST].frac & 32767);
    j.sqrt_lambda = P->sqrt_lambda;
    uint8_t org8[64 * 64];
    for (int y = 0; y < n; y++)
      for (int x = 0; x < n; x++) org8[y * n + x] = (uint8_t)*yaddr(org, 0, tpu.x0[0] + x, tpu.y0[0] + y);
    hvx_intra_search_result sr;
    hvxo_intra_search(org8, raw, &j, P->entropy_bits, &sr);
    const int nfull = sr.n_cand;
    int best_mode = 0, second_mode = -1;
    uint32_t best_dist = 0;
    double best_cost = MAX_DOUBLE, second_cost = MAX_DOUBLE;
    const int np_pu = tu_nparts(&tpu, 0);
    for (int m = 0; m < nfull; m++) {
      const int mode = sr.cand[m];
      for (int i = 0; i < np_pu; i++) cu->p[poff + i].idir[0] = (uint8_t)mode;
      e->cur = &e->goon;
      load(e->cur, &e->rd[depth][CI_CURR_BEST]);
      uint32_t d = 0;
      double c = 0.0;
      recur_intra_luma_qt(e, cu, org, pred, resi, &d, 1, &c, &tpu);
      if (c < best_cost) {
        second_mode = best_mode; second_cost = best_cost;
        best_mode = mode; best_dist = d; best_cost = c;
        set_intra_result_luma(e, cu, reco, &tpu);
        for (int i = 0; i < np_pu; i++) {
          e->tmp_tridx[i] = (uint8_t)cu->p[poff + i].tr_idx;
          for (int k = 0; k < 3; k++) { e->tmp_cbf[k][i] = cu->p[poff + i].cbf[k]; e->tmp_ts[k][i] = cu->p[poff + i].ts[k]; }
        }
      } else if (c < second_cost) {
        second_mode = mode; second_cost = c;
      }
    }
    /* HHI_RQT_INTRA_SPEEDUP_MOD is off: one full-tree pass on the best mode */
    (void)second_mode;
    {
      const int mode = best_mode;
      for (int i = 0; i < np_pu; i++) cu->p[poff + i].idir[0] = (uint8_t)mode;
      load(e->cur, &e->rd[depth][CI_CURR_BEST]);
      uint32_t d = 0;
      double c = 0.0;
      recur_intra_luma_qt(e, cu, org, pred, resi, &d, 0, &c, &tpu);
      if (c < best_cost) {
        best_mode = mode; best_dist = d; best_cost = c;
        set_intra_result_luma(e, cu, reco, &tpu);
        for (int i = 0; i < np_pu; i++) {
          e->tmp_tridx[i] = (uint8_t)cu->p[poff + i].tr_idx;
          for (int k = 0; k < 3; k++) { e->tmp_cbf[k][i] = cu->p[poff + i].cbf[k]; e->tmp_ts[k][i] = cu->p[poff + i].ts[k]; }
        }
      }
    }
    overall_dist += best_dist;
    for (int i = 0; i < np_pu; i++) {
      cu->p[poff + i].tr_idx = (int8_t)e->tmp_tridx[i];
      for (int k = 0; k < 3; k++) { cu->p[poff + i].cbf[k] = e->tmp_cbf[k][i]; cu->p[poff + i].ts[k] = e->tmp_ts[k][i]; }
    }
    if (init_trd && tpu.section < 3) {
      for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
          *rec_at(e, 0, cu->x + tpu.x0[0] + x, cu->y + tpu.y0[0] + y) = *yaddr(reco, 0, tpu.x0[0] + x, tpu.y0[0] + y);
    }
    for (int i = 0; i < np_pu; i++) cu->p[poff + i].idir[0] = (uint8_t)best_mode;
  } while (init_trd && tu_next(&tpu, &tcu));
  if (init_trd) {
    int cy = 0, cb = 0, cr = 0;
    for (int p = 0; p < 4; p++) {
      cy |= cbf_at(&cu->p[p * qnp], 0, 1);
      cb |= cbf_at(&cu->p[p * qnp], 1, 1);
      cr |= cbf_at(&cu->p[p * qnp], 2, 1);
    }
    for (int i = 0; i < 4 * qnp; i++) { cu->p[i].cbf[0] |= (uint8_t)cy; cu->p[i].cbf[1] |= (uint8_t)cb; cu->p[i].cbf[2] |= (uint8_t)cr; }
  }
  load(e->cur, &e->rd[depth][CI_CURR_BEST]);
  cu->dist = overall_dist;
}

static void recur_intra_chroma_qt(hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *pred, yuv_t *resi, uint32_t *dist, const tu_t *t) {
  const int rel = tu_abs_rel(t), trd = tu_depth_rel(t);
  const int trmode = cu->p[rel].tr_idx;
  if (trmode == trd) {
    if (!tu_proc(t, 1)) return;
    const int full_depth = tu_depth_total(t);
    int check_ts = t->w[1] <= 4;
    if (check_ts) { /* TransformSkipFast: luma 4x4 TUs and at least one luma TS */
      check_ts &= t->w[0] <= 4;
      if (check_ts) {
        int nb = 0;
        const int maxp = rel + (t->all[1] ? 1 : 4);
        for (int i = rel; i < maxp; i++) nb += cu->p[i].ts[0];
        check_ts &= nb > 0;
      }
    }
    for (int c = 1; c < 3; c++) {
      load(&e->rd[full_depth][CI_QT_TRAFO_ROOT], e->cur);
      const int crel = tu_abs_rel_c(t, c), np = tu_nparts(t, c);
      double single_cost = MAX_DOUBLE;
      int best_id = 0, best_ts = 0, single_cbf = 0;
      uint32_t single_dist = 0;
      const int total = check_ts ? 2 : 1;
      int cur_id = 0;
      for (int tsm = 0; tsm < total; tsm++) {
        set_ts_range(cu, c, crel, np, tsm);
        cur_id++;
        const int one = total == 1, last = cur_id == total;
        const int sl = one ? 0 : (tsm == 0 ? 1 : 2);
        uint32_t dtmp = 0;
        double ctmp = 0;
        intra_coding_tu(e, cu, org, pred, resi, &dtmp, c, t, sl);
        const int cbf = cbf_at(&cu->p[crel], c, trd);
        if (tsm == 1 && cbf == 0) ctmp = MAX_DOUBLE;
        else if (!one) {
          reset_bits(e);
          enc_coeff_qt(e, cu, t, c);
          ctmp = rd_cost(e, written_bits(e), dtmp);
        }
        if (ctmp < single_cost) {
          single_cost = ctmp; single_dist = dtmp; best_ts = tsm; best_id = cur_id; single_cbf = cbf;
          if (!one && !last) {
            intra_store(e, c, t);
            load(&e->rd[full_depth][CI_TEMP_BEST], e->cur);
          }
        }
        if (!one && !last) load(e->cur, &e->rd[full_depth][CI_QT_TRAFO_ROOT]);
      }
      if (best_id < total) {
        intra_load(e, cu, c, t);
        set_cbf_range(cu, c, crel, np, single_cbf << trd);
        load(e->cur, &e->rd[full_depth][CI_TEMP_BEST]);
      }
      set_ts_range(cu, c, crel, np, best_ts);
      *dist += single_dist;
    }
  } else {
    int split_cbf[3] = {0, 0, 0};
    tu_t ch;
    tu_child(&ch, t, 0);
    const int trd_child = tu_depth_rel(&ch);
    do {
      recur_intra_chroma_qt(e, cu, org, pred, resi, dist, &ch);
      const int sub = tu_abs_rel(&ch);
      for (int c = 1; c < 3; c++) split_cbf[c] |= cbf_at(&cu->p[sub], c, trd_child);
    } while (tu_next(&ch, t));
    for (int c = 1; c < 3; c++)
      if (split_cbf[c])
        for (int i = 0; i < t->step; i++) cu->p[rel + i].cbf[c] |= (uint8_t)(1 << trd);
  }
}
/* xSetIntraResultChromaQT (:2124) */
static void set_intra_result_chroma(hm_enc *e, hm_cu *cu, yuv_t *reco, const tu_t *t) {
  if (!tu_proc(t, 1)) return;
  const int rel = tu_abs_rel(t);
  if (cu->p[rel].tr_idx == tu_depth_rel(t)) {
    const int layer = qt_layer(t->log2), w = t->w[1];
    for (int c = 1; c < 3; c++) {
      memcpy(cu->coef[c] + t->off[c], e->qt_coef[c][layer] + t->off[c], sizeof(int32_t) * w * w);
      for (int y = 0; y < w; y++)
        memcpy(yaddr(reco, c, t->x0[c], t->y0[c] + y), yaddr(&e->qt_yuv[layer], c, t->x0[c], t->y0[c] + y), sizeof(int16_t) * w);
    }
  } else {
    tu_t ch;
    tu_child(&ch, t, 0);
    do set_intra_result_chroma(e, cu, reco, &ch); while (tu_next(&ch, t));
  }
}
static void est_intra_pred_chroma_qt(hm_enc *e, hm_cu *cu, yuv_t *org, yuv_t *pred, yuv_t *resi, yuv_t *reco) {
  const int depth = cu->depth;
  tu_t t;
  tu_root(&t, cu, 0);
  const int np = t.step;
  int best_mode = 0;
  uint32_t best_dist = 0;
  double best_cost = MAX_DOUBLE;
  int modes[5] = {0, 26, 10, 1, DM_CHROMA_IDX};
  const int lm = cu->p[0].idir[0];
  for (int i = 0; i < 4; i++) if (lm == modes[i]) { modes[i] = 34; break; }
  uint8_t save_cbf[3][256], save_ts[3][256];
  for (int m = 0; m < 5; m++) {
    e->cur = &e->goon;
    load(e->cur, &e->rd[depth][CI_CURR_BEST]);
    uint32_t d = 0;
    for (int i = 0; i < np; i++) cu->p[i].idir[1] = (uint8_t)modes[m];
    recur_intra_chroma_qt(e, cu, org, pred, resi, &d, &t);
    load(e->cur, &e->rd[depth][CI_CURR_BEST]); /* TransformSkip on */
    const uint32_t b = intra_bits_qt(e, cu, &t, 0, 1);
    const double c = rd_cost(e, b, d);
    if (c < best_cost) {
      best_cost = c; best_dist = d; best_mode = modes[m];
      set_intra_result_chroma(e, cu, reco, &t);
      for (int k = 1; k < 3; k++)
        for (int i = 0; i < np; i++) { save_cbf[k][i] = cu->p[i].cbf[k]; save_ts[k][i] = cu->p[i].ts[k]; }
    }
  }
  for (int k = 1; k < 3; k++)
    for (int i = 0; i < np; i++) { cu->p[i].cbf[k] = save_cbf[k][i]; cu->p[i].ts[k] = save_ts[k][i]; }
  for (int i = 0; i < np; i++) cu->p[i].idir[1] = (uint8_t)best_mode;
  cu->dist += best_dist;
  load(e->cur, &e->rd[depth][CI_CURR_BEST]);
}

/* ============================================================================================
 * TEncCu: xCheckBestMode (TEncCu.cpp:1444), xCheckRDCostMerge2Nx2N (:1166), xCheckRDCostInter
 * (:1291), xCheckRDCostIntra (:1330), deriveTestModeAMP (:274), xCompressCU (:349)
 * ========================================================================================== */
static void check_best_mode(hm_enc *e, int depth) {
  if (e->temp[depth]->cost < e->best[depth]->cost) {
    hm_cu *t = e->best[depth]; e->best[depth] = e->temp[depth]; e->temp[depth] = t;
    yuv_t *y = e->pred_best[depth]; e->pred_best[depth] = e->pred_temp[depth]; e->pred_temp[depth] = y;
    y = e->reco_best[depth]; e->reco_best[depth] = e->reco_temp[depth]; e->reco_temp[depth] = y;
    load(&e->rd[depth][CI_NEXT_BEST], &e->rd[depth][CI_TEMP_BEST]);
  }
}
static void reinit_temp(hm_enc *e, int depth) { cu_init_est(e->temp[depth], e->slice_qp); }

static void check_rd_merge2nx2n(hm_enc *e, int depth) {
  hm_cu *tmp = e->temp[depth];
  mvfield_t f[10];
  int dirs[5];
  cu_set_all(tmp, F_PART, SIZE_2Nx2N);
  const int n = merge_candidates(e, tmp, SIZE_2Nx2N, 0, f, dirs);
  int buf[5] = {0, 0, 0, 0, 0};
  int best_is_skip = 0;
  for (int nores = 0; nores < 2; nores++) {
    for (int m = 0; m < n; m++) {
      if (nores == 1 && buf[m] == 1) continue;
      if (best_is_skip && nores == 0) continue;
      tmp = e->temp[depth];
      cu_set_all(tmp, F_PRED, MODE_INTER);
      cu_set_all(tmp, F_PART, SIZE_2Nx2N);
      for (int i = 0; i < tmp->nparts; i++) {
        tmp->p[i].merge = 1;
        tmp->p[i].merge_idx = (int8_t)m;
        tmp->p[i].inter_dir = (int8_t)dirs[m];
        for (int l = 0; l < 2; l++) {
          tmp->p[i].mv[l][0] = f[2 * m + l].mv[0];
          tmp->p[i].mv[l][1] = f[2 * m + l].mv[1];
          tmp->p[i].ref[l] = (int8_t)f[2 * m + l].ref;
        }
      }
      mc_cu(e, tmp, e->pred_temp[depth]);
      enc_res_rd_inter(e, tmp, e->orig[depth], e->pred_temp[depth], e->resi_temp[depth], e->resi_best[depth], e->reco_temp[depth],
                       nores != 0);
      if (nores == 0 && !cu_qt_root_cbf(tmp, 0)) buf[m] = 1;
      check_best_mode(e, depth);
      reinit_temp(e, depth);
      if (!best_is_skip) best_is_skip = !cu_qt_root_cbf(e->best[depth], 0); /* FDM */
    }
  }
}
static void check_rd_inter(hm_enc *e, int depth, int ps, int use_mrg) {
  hm_cu *tmp = e->temp[depth];
  cu_set_all(tmp, F_PART, ps);
  cu_set_all(tmp, F_PRED, MODE_INTER);
  tmp->merge_amp = 1;
  pred_inter_search(e, tmp, e->orig[depth], e->pred_temp[depth], use_mrg);
  enc_res_rd_inter(e, tmp, e->orig[depth], e->pred_temp[depth], e->resi_temp[depth], e->resi_best[depth], e->reco_temp[depth], 0);
  tmp->cost = cu_cost(e, tmp, tmp->bits, tmp->dist);
  check_best_mode(e, depth);
}
static void check_rd_intra(hm_enc *e, int depth, int ps) {
  hm_cu *tmp = e->temp[depth];
  cu_set_all(tmp, F_SKIP, 0);
  cu_set_all(tmp, F_PART, ps);
  cu_set_all(tmp, F_PRED, MODE_INTRA);
  est_intra_pred_luma_qt(e, tmp, e->orig[depth], e->pred_temp[depth], e->resi_temp[depth], e->reco_temp[depth]);
  yuv_to_pic_comp(e, e->reco_temp[depth], tmp, 0);
  est_intra_pred_chroma_qt(e, tmp, e->orig[depth], e->pred_temp[depth], e->resi_temp[depth], e->reco_temp[depth]);
  reset_bits(e);
  code_skip_flag(e, tmp, 0);
  code_pred_mode(e, tmp, 0);
  code_part_size(e, tmp, 0, depth);
  encode_pred_info(e, tmp, 0);
  encode_coeff(e, tmp, 0);
  load(&e->rd[depth][CI_TEMP_BEST], e->cur);
  tmp->bits = written_bits(e);
  cu_measure_ssim(e, tmp, e->orig[depth], e->reco_temp[depth]);
  tmp->cost = cu_cost(e, tmp, tmp->bits, tmp->dist);
  check_best_mode(e, depth);
}
static void derive_test_mode_amp(const hm_cu *best, int parent_ps, int *hor, int *ver, int *mhor, int *mver) {
  const int ps = best->p[0].part;
  if (ps == SIZE_2NxN) *hor = 1;
  else if (ps == SIZE_Nx2N) *ver = 1;
  else if (ps == SIZE_2Nx2N && !best->p[0].merge && !best->p[0].skip) { *hor = 1; *ver = 1; }
  if (parent_ps >= SIZE_2NxnU && parent_ps <= SIZE_nRx2N) { *mhor = 1; *mver = 1; }
  if (parent_ps == SIZE_NONE) {
    if (ps == SIZE_2NxN) *mhor = 1;
    else if (ps == SIZE_Nx2N) *mver = 1;
  }
  if (ps == SIZE_2Nx2N && !best->p[0].skip) { *mhor = 1; *mver = 1; }
  if (best->width == 64) { *hor = 0; *ver = 0; }
}

static void compress_cu(hm_enc *e, int depth, int parent_ps) {
  const hvxo_hm_pic *P = e->pic;
  hm_cu *best = e->best[depth];
  copy_org_to_yuv(e, e->orig[depth], best);
  int sub_branch = 1, do_not_block = 1;
  const int rx = best->x + best->width - 1, by = best->y + best->width - 1;
  int boundary = 0;
  const int qp = e->slice_qp;
  if (rx < P->w && by < P->h) {
    reinit_temp(e, depth);
    if (P->slice_type != I_SLICE) {
      check_rd_merge2nx2n(e, depth);
      reinit_temp(e, depth);
      check_rd_inter(e, depth, SIZE_2Nx2N, 0);
      reinit_temp(e, depth);
      do_not_block = cu_qt_root_cbf(e->best[depth], 0) != 0; /* CFM off: getUseCbfFastMode false */
      do_not_block = 1;
    }
    reinit_temp(e, depth);
    if (P->slice_type != I_SLICE) {
      if (do_not_block) {
        check_rd_inter(e, depth, SIZE_Nx2N, 0);
        reinit_temp(e, depth);
      }
      if (do_not_block) {
        check_rd_inter(e, depth, SIZE_2NxN, 0);
        reinit_temp(e, depth);
      }
      if (P->amp && depth < 3) {
        int hor = 0, ver = 0, mhor = 0, mver = 0;
        derive_test_mode_amp(e->best[depth], parent_ps, &hor, &ver, &mhor, &mver);
        if (hor) {
          check_rd_inter(e, depth, SIZE_2NxnU, 0); reinit_temp(e, depth);
          check_rd_inter(e, depth, SIZE_2NxnD, 0); reinit_temp(e, depth);
        } else if (mhor) {
          check_rd_inter(e, depth, SIZE_2NxnU, 1); reinit_temp(e, depth);
          check_rd_inter(e, depth, SIZE_2NxnD, 1); reinit_temp(e, depth);
        }
        if (ver) {
          check_rd_inter(e, depth, SIZE_nLx2N, 0); reinit_temp(e, depth);
          check_rd_inter(e, depth, SIZE_nRx2N, 0); reinit_temp(e, depth);
        } else if (mver) {
          check_rd_inter(e, depth, SIZE_nLx2N, 1); reinit_temp(e, depth);
          check_rd_inter(e, depth, SIZE_nRx2N, 1); reinit_temp(e, depth);
        }
      }
    }
    best = e->best[depth];
    if (P->slice_type == I_SLICE || (best->p[0].cbf[0] || best->p[0].cbf[1] || best->p[0].cbf[2])) {
      check_rd_intra(e, depth, SIZE_2Nx2N);
      reinit_temp(e, depth);
      if (depth == 3 && e->temp[depth]->width > 4) {
        check_rd_intra(e, depth, SIZE_NxN);
        reinit_temp(e, depth);
      }
    }
    best = e->best[depth];
    e->cur = &e->goon;
    load(e->cur, &e->rd[depth][CI_NEXT_BEST]);
    reset_bits(e);
    code_split_flag(e, best, 0, depth);
    best->bits += written_bits(e);
    best->cost = cu_cost(e, best, best->bits, best->dist);
    load(&e->rd[depth][CI_NEXT_BEST], e->cur);
    sub_branch = 1; /* ECU off */
  } else boundary = 1;

  reinit_temp(e, depth);
  if (sub_branch && depth < 3) {
    const int nd = depth + 1;
    hm_cu *tmp = e->temp[depth];
    for (int k = 0; k < 4; k++) {
      cu_init_sub(e->best[nd], tmp, k, nd, qp);
      cu_init_sub(e->temp[nd], tmp, k, nd, qp);
      hm_cu *sb = e->best[nd];
      if (sb->x < P->w && sb->y < P->h) {
        if (k == 0) load(&e->rd[nd][CI_CURR_BEST], &e->rd[depth][CI_CURR_BEST]);
        else load(&e->rd[nd][CI_CURR_BEST], &e->rd[nd][CI_NEXT_BEST]);
        compress_cu(e, nd, e->best[depth]->p[0].pred != MODE_INTER ? SIZE_NONE : e->best[depth]->p[0].part);
        tmp = e->temp[depth];
        cu_copy_part_from(tmp, e->best[nd], k, nd);
        yuv_child_to_parent(e->reco_temp[depth], e->reco_best[nd], k, sb->width);
      } else {
        cu_copy_to_pic(e, sb);
        tmp = e->temp[depth];
        cu_copy_part_from(tmp, sb, k, nd);
      }
    }
    tmp = e->temp[depth];
    e->cur = &e->goon;
    load(e->cur, &e->rd[nd][CI_NEXT_BEST]);
    if (!boundary) {
      reset_bits(e);
      code_split_flag(e, tmp, 0, depth);
      tmp->bits += written_bits(e);
    }
    tmp->cost = cu_cost(e, tmp, tmp->bits, tmp->dist);
    load(&e->rd[depth][CI_TEMP_BEST], e->cur);
    check_best_mode(e, depth);
  }
  cu_copy_to_pic(e, e->best[depth]);
  yuv_to_pic(e, e->reco_best[depth], e->best[depth]);
}

/* ============================================================================================
 * TEncCu::xEncodeCU (TEncCu.cpp:920) under the counter: the true CTU coding whose context
 * states start the next CTU (TEncSlice.cpp:821-831).
 * ========================================================================================== */
static void encode_cu(hm_enc *e, hm_cu *ctu, int rel, int depth, int last_ctu_in_slice) {
  const hvxo_hm_pic *P = e->pic;
  const int r = Z2R[rel];
  const int lx = e->ctu_x * 64 + RPX(r), ty = e->ctu_y * 64 + RPY(r);
  const int sz = 64 >> depth;
  const int rx = lx + sz - 1, by = ty + sz - 1;
  int boundary = 0;
  if (rx < P->w && by < P->h) code_split_flag(e, ctu, rel, depth);
  else boundary = 1;
  if ((depth < ctu->p[rel].depth && depth < 3) || boundary) {
    const int q = (256 >> (2 * depth)) >> 2;
    for (int k = 0; k < 4; k++) {
      const int sub = rel + k * q, rs = Z2R[sub];
      if (e->ctu_x * 64 + RPX(rs) < P->w && e->ctu_y * 64 + RPY(rs) < P->h) encode_cu(e, ctu, sub, depth + 1, last_ctu_in_slice);
    }
    return;
  }
  code_skip_flag(e, ctu, rel);
  if (ctu->p[rel].skip) {
    code_merge_index(e, ctu, rel);
  } else {
    code_pred_mode(e, ctu, rel);
    code_part_size(e, ctu, rel, depth);
    encode_pred_info(e, ctu, rel);
    if (ctu->p[rel].pred != MODE_INTRA && !(ctu->p[rel].merge && ctu->p[rel].part == SIZE_2Nx2N))
      cbin(e, X_ROOT_CBF, cu_qt_root_cbf(ctu, rel));
    if (ctu->p[rel].pred == MODE_INTRA || cu_qt_root_cbf(ctu, rel)) {
      /* TComTURecurse(pcCU, uiAbsPartIdx, uiDepth) over the CTU object: a CU-relative view */
      static _Thread_local hm_cu view;
      view.depth = depth; view.zidx = rel; view.width = sz; view.nparts = 256 >> (2 * depth);
      view.x = lx; view.y = ty; view.ctu = e->ctu_addr;
      memcpy(view.p, &ctu->p[rel], sizeof(hm_part) * view.nparts);
      const int off = rel * 16;
      memcpy(view.coef[0], ctu->coef[0] + off, sizeof(int32_t) * sz * sz);
      memcpy(view.coef[1], ctu->coef[1] + (off >> 2), sizeof(int32_t) * (sz * sz >> 2));
      memcpy(view.coef[2], ctu->coef[2] + (off >> 2), sizeof(int32_t) * (sz * sz >> 2));
      tu_t t;
      tu_root(&t, &view, 0);
      encode_transform(e, &view, &t);
    }
  }
  /* finishCU (TEncCu.cpp:885) with isLastSubCUOfCtu (TComDataCU.cpp:405): the terminating bin
   * after the CTU's last CU, unless the CTU ends the slice */
  const int ex = lx + sz, ey = ty + sz;
  if ((ex % 64 == 0 || ex == P->w) && (ey % 64 == 0 || ey == P->h) && !last_ctu_in_slice) ctrm(e, 0);
}

/* ============================================================================================
 * API
 * ========================================================================================== */
static hm_enc *enc_new(void) {
  hm_enc *e = (hm_enc *)calloc(1, sizeof(hm_enc));
  for (int d = 0; d < 4; d++) {
    e->best[d] = &e->cu_store[0][d];
    e->temp[d] = &e->cu_store[1][d];
    e->orig[d] = &e->yuv_store[0][d];
    e->pred_best[d] = &e->yuv_store[1][d];
    e->pred_temp[d] = &e->yuv_store[2][d];
    e->resi_best[d] = &e->yuv_store[3][d];
    e->resi_temp[d] = &e->yuv_store[4][d];
    e->reco_best[d] = &e->yuv_store[5][d];
    e->reco_temp[d] = &e->yuv_store[6][d];
  }
  return e;
}

void hvxo_hm_compress_ctu(const hvxo_hm_pic *pic, hvxo_hm_ctu_data *ctus, int16_t *const *rec, const int *rec_stride,
                          int ctu_addr, const hvxo_hm_coder *entry, const int16_t *int2n, hvxo_hm_coder *after_encode) {
  hvxo_hm_compress_ctu_slice(pic, ctus, rec, rec_stride, ctu_addr, 0, pic->w_ctus * pic->h_ctus - 1, entry, int2n, NULL,
                             after_encode);
}

void hvxo_hm_compress_ctu_slice(const hvxo_hm_pic *pic, hvxo_hm_ctu_data *ctus, int16_t *const *rec, const int *rec_stride,
                                int ctu_addr, int slice_start, int slice_end, const hvxo_hm_coder *entry,
                                const int16_t *int2n, int16_t *int2n_out, hvxo_hm_coder *after_encode) {
  tables_init();
  hm_enc *e = enc_new();
  e->pic = pic;
  e->ctus = ctus;
  for (int c = 0; c < 3; c++) { e->rec[c] = rec[c]; e->rs[c] = rec_stride[c]; }
  e->ctu_addr = ctu_addr;
  e->ctu_x = ctu_addr % pic->w_ctus;
  e->ctu_y = ctu_addr / pic->w_ctus;
  e->slice_qp = pic->qp;
  e->slice_start = slice_start;
  e->slice_end = slice_end;
  memcpy(e->int2n, int2n, sizeof(e->int2n));
  /* TComDataCU::initCtu (TComDataCU.cpp:434) of the picture's CTU and of the depth-0 best/temp CUs */
  hvxo_hm_ctu_data *d = &ctus[ctu_addr];
  hm_cu *c0 = e->best[0];
  c0->depth = 0; c0->width = 64; c0->nparts = 256; c0->zidx = 0;
  c0->x = e->ctu_x * 64; c0->y = e->ctu_y * 64; c0->ctu = ctu_addr;
  cu_init_est(c0, pic->qp);
  e->temp[0]->depth = 0; e->temp[0]->width = 64; e->temp[0]->nparts = 256; e->temp[0]->zidx = 0;
  e->temp[0]->x = c0->x; e->temp[0]->y = c0->y; e->temp[0]->ctu = ctu_addr;
  cu_init_est(e->temp[0], pic->qp);
  memcpy(d->p, c0->p, sizeof(d->p));
  memset(d->coef, 0, sizeof(d->coef));
  d->bits = 0; d->dist = 0; d->cost = MAX_DOUBLE;
  load(&e->rd[0][CI_CURR_BEST], entry);
  e->cur = &e->goon;
  load(e->cur, &e->rd[0][CI_CURR_BEST]); /* TEncSlice.cpp:764 */
  compress_cu(e, 0, SIZE_NONE);
  if (after_encode) {
    /* encodeCtu on m_pppcRDSbacCoder[0][CI_CURR_BEST] after resetBits (TEncSlice.cpp:821-828); the
     * decision does not write that coder, so it still holds the entry state */
    e->cur = &e->rd[0][CI_CURR_BEST];
    load(e->cur, entry);
    reset_bits(e);
    static _Thread_local hm_cu view;
    view.depth = 0; view.zidx = 0; view.width = 64; view.nparts = 256;
    view.x = e->ctu_x * 64; view.y = e->ctu_y * 64; view.ctu = ctu_addr;
    memcpy(view.p, d->p, sizeof(d->p));
    memcpy(view.coef, d->coef, sizeof(d->coef));
    encode_cu(e, &view, 0, 0, ctu_addr == slice_end);
    *after_encode = *e->cur;
  }
  if (int2n_out) memcpy(int2n_out, e->int2n, sizeof(e->int2n));
  free(e);
}

/* the cu_capture.cpp pic_i32 / pic_f64 fields */
enum {
  P_W, P_H, P_POC, P_SLICE_TYPE, P_QP, P_NREF0, P_NREF1, P_REFPOC0, P_REFPOC1 = P_REFPOC0 + 4,
  P_REFPIC0 = P_REFPOC1 + 4, P_REFPIC1 = P_REFPIC0 + 4, P_COL_FROM_L0 = P_REFPIC1 + 4, P_COL_REF_IDX, P_CHECK_LDC,
  P_TMVP, P_MAX_MERGE, P_COL_POC, P_COL_NREF0, P_COL_NREF1, P_COL_REFPOC0, P_COL_REFPOC1 = P_COL_REFPOC0 + 4,
  P_CHROMA_QP_CB = P_COL_REFPOC1 + 4, P_CHROMA_QP_CR, P_FIRST_CTU, P_NCTU, P_LAMBDA_MOTION, P_CABAC_TABLE,
  P_COL_VALID, P_NFIELDS
};
enum { F_LAMBDA, F_SQRT_LAMBDA, F_WEIGHT_CB, F_WEIGHT_CR, F_TQ_LAMBDA_Y, F_TQ_LAMBDA_CB, F_TQ_LAMBDA_CR };

/* a padded copy of an 8-bit plane with its border extended (TComPicYuv::extendPicBorder) */
static void pad_plane16(const uint8_t *src, int w, int h, int m, int16_t *dst, int ds) {
  for (int y = -m; y < h + m; y++) {
    const int sy = y < 0 ? 0 : y >= h ? h - 1 : y;
    for (int x = -m; x < w + m; x++) {
      const int sx = x < 0 ? 0 : x >= w ? w - 1 : x;
      dst[(y + m) * ds + x + m] = src[sy * w + sx];
    }
  }
}
static void pad_plane8(const uint8_t *src, int w, int h, int m, uint8_t *dst, int ds) {
  for (int y = -m; y < h + m; y++) {
    const int sy = y < 0 ? 0 : y >= h ? h - 1 : y;
    for (int x = -m; x < w + m; x++) {
      const int sx = x < 0 ? 0 : x >= w ? w - 1 : x;
      dst[(y + m) * ds + x + m] = src[sy * w + sx];
    }
  }
}

/* the picture the cu_capture.cpp arrays describe: parameters, 16-bit originals, padded references */
typedef struct {
  hvxo_hm_pic P;
  int16_t *org16[3];
  int16_t **planes16, **bufs16;
  uint8_t **planes8, **bufs8;
  int n_refpics;
} pic_buf;
static void pic_setup(pic_buf *B, const int32_t *pi, const double *pf, const uint8_t *org, const uint8_t *refpics, int n_refpics,
                      const int16_t *col_field, const int32_t *entropy_bits) {
  memset(B, 0, sizeof(*B));
  B->n_refpics = n_refpics;
  const int w = pi[P_W], h = pi[P_H], wc = (w + 63) / 64, hc = (h + 63) / 64;
  const int M = 80, MC = 40;
  B->P.w = w; B->P.h = h; B->P.w_ctus = wc; B->P.h_ctus = hc;
  B->P.poc = pi[P_POC]; B->P.slice_type = pi[P_SLICE_TYPE]; B->P.qp = pi[P_QP];
  B->P.nref[0] = pi[P_NREF0]; B->P.nref[1] = pi[P_NREF1];
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < 4; i++) {
      B->P.ref_poc[l][i] = pi[(l ? P_REFPOC1 : P_REFPOC0) + i];
      B->P.ref_plane_idx[l][i] = pi[(l ? P_REFPIC1 : P_REFPIC0) + i];
      B->P.col_ref_poc[l][i] = pi[(l ? P_COL_REFPOC1 : P_COL_REFPOC0) + i];
    }
  B->P.chroma_qp[0] = pi[P_CHROMA_QP_CB]; B->P.chroma_qp[1] = pi[P_CHROMA_QP_CR];
  B->P.max_merge = pi[P_MAX_MERGE]; B->P.tmvp = pi[P_TMVP]; B->P.check_ldc = pi[P_CHECK_LDC];
  B->P.col_from_l0 = pi[P_COL_FROM_L0]; B->P.col_valid = pi[P_COL_VALID]; B->P.col_poc = pi[P_COL_POC];
  B->P.col_field = col_field;
  B->P.lambda = pf[F_LAMBDA]; B->P.sqrt_lambda = pf[F_SQRT_LAMBDA];
  B->P.chroma_weight[0] = pf[F_WEIGHT_CB]; B->P.chroma_weight[1] = pf[F_WEIGHT_CR];
  B->P.tq_lambda[0] = pf[F_TQ_LAMBDA_Y]; B->P.tq_lambda[1] = pf[F_TQ_LAMBDA_CB]; B->P.tq_lambda[2] = pf[F_TQ_LAMBDA_CR];
  B->P.lambda_motion = (uint32_t)pi[P_LAMBDA_MOTION];
  hvxo_hm_derive_lists(&B->P);
  B->P.search_range = 64;
  B->P.bipred_range = 4;
  B->P.amp = 1;
  B->P.entropy_bits = entropy_bits;
  /* original planes */
  const size_t ysz = (size_t)w * h, csz = ysz / 4;
  for (int c = 0; c < 3; c++) {
    const size_t sz = c ? csz : ysz;
    B->org16[c] = (int16_t *)malloc(sizeof(int16_t) * sz);
    const uint8_t *s8 = org + (c == 0 ? 0 : c == 1 ? ysz : ysz + csz);
    for (size_t i = 0; i < sz; i++) B->org16[c][i] = s8[i];
    B->P.org[c] = B->org16[c];
    B->P.org_stride[c] = c ? w / 2 : w;
  }
  B->P.org8 = org;
  B->P.org8_stride = w;
  /* reference planes, padded */
  const int s16y = w + 2 * M, s16c = w / 2 + 2 * MC;
  B->planes16 = (int16_t **)calloc((size_t)3 * (n_refpics ? n_refpics : 1), sizeof(int16_t *));
  B->planes8 = (uint8_t **)calloc((size_t)(n_refpics ? n_refpics : 1), sizeof(uint8_t *));
  B->bufs16 = (int16_t **)calloc((size_t)3 * (n_refpics ? n_refpics : 1), sizeof(int16_t *));
  B->bufs8 = (uint8_t **)calloc((size_t)(n_refpics ? n_refpics : 1), sizeof(uint8_t *));
  for (int r = 0; r < n_refpics; r++) {
    const uint8_t *base = refpics + (size_t)r * (ysz + 2 * csz);
    for (int c = 0; c < 3; c++) {
      const int cw = c ? w / 2 : w, ch = c ? h / 2 : h, m = c ? MC : M, st = c ? s16c : s16y;
      B->bufs16[3 * r + c] = (int16_t *)malloc(sizeof(int16_t) * (size_t)st * (ch + 2 * m));
      pad_plane16(base + (c == 0 ? 0 : c == 1 ? ysz : ysz + csz), cw, ch, m, B->bufs16[3 * r + c], st);
      B->planes16[3 * r + c] = B->bufs16[3 * r + c] + m * st + m;
    }
    B->bufs8[r] = (uint8_t *)malloc((size_t)s16y * (h + 2 * M));
    pad_plane8(base, w, h, M, B->bufs8[r], s16y);
    B->planes8[r] = B->bufs8[r] + M * s16y + M;
  }
  B->P.ref_planes16 = (const int16_t *const *)B->planes16;
  B->P.ref_stride16[0] = s16y; B->P.ref_stride16[1] = s16c;
  B->P.ref_planes8 = (const uint8_t *const *)B->planes8;
  B->P.ref_stride8 = s16y;
}
static void pic_free(pic_buf *B) {
  for (int c = 0; c < 3; c++) free(B->org16[c]);
  for (int r = 0; r < 3 * B->n_refpics; r++) free(B->bufs16[r]);
  for (int r = 0; r < B->n_refpics; r++) free(B->bufs8[r]);
  free(B->planes16); free(B->planes8); free(B->bufs16); free(B->bufs8);
}

int hvxo_hm_replay_picture(const int32_t *pi, const double *pf, const uint8_t *org, const uint8_t *refpics,
                           const int32_t *refpic_poc, int n_refpics, const int16_t *col_field, const int32_t *entropy_bits,
                           const uint8_t *ctu_states, const int64_t *ctu_frac, const int16_t *ctu_int2n,
                           const int16_t *hm_parts, const int32_t *hm_coef, const uint8_t *hm_recon, int mode,
                           int slice_ctus, int16_t *out_parts, int32_t *out_coef, uint8_t *out_recon, double *out_cost,
                           uint32_t *out_bits_dist, uint8_t *out_states, int64_t *out_frac) {
  return hvxo_hm_replay_picture_rd(pi, pf, org, refpics, refpic_poc, n_refpics, col_field, entropy_bits, ctu_states, ctu_frac,
                                   ctu_int2n, hm_parts, hm_coef, hm_recon, mode, slice_ctus, 0, 0.0, out_parts, out_coef,
                                   out_recon, out_cost, out_bits_dist, out_states, out_frac);
}
int hvxo_hm_replay_picture_rd(const int32_t *pi, const double *pf, const uint8_t *org, const uint8_t *refpics,
                              const int32_t *refpic_poc, int n_refpics, const int16_t *col_field, const int32_t *entropy_bits,
                              const uint8_t *ctu_states, const int64_t *ctu_frac, const int16_t *ctu_int2n,
                              const int16_t *hm_parts, const int32_t *hm_coef, const uint8_t *hm_recon, int mode,
                              int slice_ctus, int rd_metric, double lambda_ssim, int16_t *out_parts, int32_t *out_coef,
                              uint8_t *out_recon, double *out_cost, uint32_t *out_bits_dist, uint8_t *out_states,
                              int64_t *out_frac) {
  return hvxo_hm_replay_picture_stv(pi, pf, org, refpics, refpic_poc, n_refpics, col_field, entropy_bits, ctu_states,
                                    ctu_frac, ctu_int2n, hm_parts, hm_coef, hm_recon, mode, slice_ctus, rd_metric,
                                    lambda_ssim, NULL, out_parts, out_coef, out_recon, out_cost, out_bits_dist, out_states,
                                    out_frac);
}
static void set_stv(hvxo_hm_pic *P, const hvxo_stv *stv) {
  P->hist = NULL; P->hist_n = 0; P->hist_stride[0] = P->hist_stride[1] = 0; P->dirs = NULL; P->dirs_stride = 0;
  if (!stv) return;
  P->hist = stv->hist;
  P->hist_n = stv->hist_n < 0 ? 0 : stv->hist_n > 25 ? 25 : stv->hist_n;
  P->hist_stride[0] = stv->hist_stride[0];
  P->hist_stride[1] = stv->hist_stride[1];
  P->dirs = stv->dirs;
  P->dirs_stride = stv->dirs_stride;
}
int hvxo_hm_replay_picture_stv(const int32_t *pi, const double *pf, const uint8_t *org, const uint8_t *refpics,
                               const int32_t *refpic_poc, int n_refpics, const int16_t *col_field, const int32_t *entropy_bits,
                               const uint8_t *ctu_states, const int64_t *ctu_frac, const int16_t *ctu_int2n,
                               const int16_t *hm_parts, const int32_t *hm_coef, const uint8_t *hm_recon, int mode,
                               int slice_ctus, int rd_metric, double lambda_ssim, const hvxo_stv *stv, int16_t *out_parts,
                               int32_t *out_coef, uint8_t *out_recon, double *out_cost, uint32_t *out_bits_dist,
                               uint8_t *out_states, int64_t *out_frac) {
  (void)refpic_poc;
  tables_init();
  const int w = pi[P_W], h = pi[P_H], wc = (w + 63) / 64, hc = (h + 63) / 64, n = wc * hc;
  pic_buf B;
  pic_setup(&B, pi, pf, org, refpics, n_refpics, col_field, entropy_bits);
  B.P.rd_metric = rd_metric;
  B.P.lambda_ssim = lambda_ssim;
  set_stv(&B.P, stv);
  const hvxo_hm_pic P = B.P;
  /* the picture's CTU data and reconstruction (whole CTUs) */
  hvxo_hm_ctu_data *ctus = (hvxo_hm_ctu_data *)calloc((size_t)n, sizeof(hvxo_hm_ctu_data));
  const int rw = wc * 64, rh = hc * 64;
  int16_t *recb[3];
  int rs[3] = {rw, rw / 2, rw / 2};
  for (int c = 0; c < 3; c++) recb[c] = (int16_t *)calloc((size_t)(c ? rw * rh / 4 : rw * rh), sizeof(int16_t));
  hvxo_hm_coder prev;
  for (int a = 0; a < n; a++) {
    hvxo_hm_coder entry;
    const int s0 = slice_ctus > 0 ? a - a % slice_ctus : 0;
    const int s1 = slice_ctus > 0 ? (s0 + slice_ctus < n ? s0 + slice_ctus : n) - 1 : n - 1;
    if (mode == 0 || a == s0) {
      memcpy(entry.st, ctu_states + (size_t)a * 202, 202);
      entry.frac = (uint64_t)ctu_frac[a];
    } else entry = prev;
    if (mode == 0 && a > 0) { /* the reference's previous CTU: data + reconstruction */
      hvxo_hm_ctu_data *q = &ctus[a - 1];
      hvxo_hm_pack_parts(q, hm_parts + (size_t)(a - 1) * 256 * HVXO_HM_PART_FIELDS);
      memcpy(q->coef[0], hm_coef + (size_t)(a - 1) * 6144, sizeof(int32_t) * 4096);
      memcpy(q->coef[1], hm_coef + (size_t)(a - 1) * 6144 + 4096, sizeof(int32_t) * 1024);
      memcpy(q->coef[2], hm_coef + (size_t)(a - 1) * 6144 + 5120, sizeof(int32_t) * 1024);
      const uint8_t *rr = hm_recon + (size_t)(a - 1) * 6144;
      const int ax = (a - 1) % wc, ay = (a - 1) / wc;
      for (int y = 0; y < 64; y++)
        for (int x = 0; x < 64; x++) recb[0][(ay * 64 + y) * rs[0] + ax * 64 + x] = rr[y * 64 + x];
      for (int c = 1; c < 3; c++)
        for (int y = 0; y < 32; y++)
          for (int x = 0; x < 32; x++) recb[c][(ay * 32 + y) * rs[c] + ax * 32 + x] = rr[4096 + (c - 1) * 1024 + y * 32 + x];
    }
    hvxo_hm_coder after;
    hvxo_hm_compress_ctu_slice(&P, ctus, recb, rs, a, s0, s1, &entry, ctu_int2n + (size_t)a * 16, NULL, &after);
    prev = after;
    if (out_states) memcpy(out_states + (size_t)a * 202, after.st, 202);
    if (out_frac) out_frac[a] = (int64_t)after.frac;
    hvxo_hm_ctu_data *q = &ctus[a];
    if (out_parts) hvxo_hm_unpack_parts(q, out_parts + (size_t)a * 256 * HVXO_HM_PART_FIELDS);
    if (out_coef) {
      memcpy(out_coef + (size_t)a * 6144, q->coef[0], sizeof(int32_t) * 4096);
      memcpy(out_coef + (size_t)a * 6144 + 4096, q->coef[1], sizeof(int32_t) * 1024);
      memcpy(out_coef + (size_t)a * 6144 + 5120, q->coef[2], sizeof(int32_t) * 1024);
    }
    if (out_cost) out_cost[a] = q->cost;
    if (out_bits_dist) { out_bits_dist[2 * a] = q->bits; out_bits_dist[2 * a + 1] = q->dist; }
    if (out_recon) {
      const int ax = a % wc, ay = a / wc;
      uint8_t *o = out_recon + (size_t)a * 6144;
      for (int y = 0; y < 64; y++)
        for (int x = 0; x < 64; x++)
          o[y * 64 + x] = (ax * 64 + x < w && ay * 64 + y < h) ? (uint8_t)recb[0][(ay * 64 + y) * rs[0] + ax * 64 + x] : 0;
      for (int c = 1; c < 3; c++)
        for (int y = 0; y < 32; y++)
          for (int x = 0; x < 32; x++)
            o[4096 + (c - 1) * 1024 + y * 32 + x] = (ax * 32 + x < w / 2 && ay * 32 + y < h / 2)
                                                        ? (uint8_t)recb[c][(ay * 32 + y) * rs[c] + ax * 32 + x]
                                                        : 0;
    }
  }
  for (int c = 0; c < 3; c++) free(recb[c]);
  pic_free(&B);
  free(ctus);
  return n;
}

/* ============================================================================================
 * Independent slice chains (the bench's HM-exact workload): SliceMode=1 slices, each chain the
 * first ctus_per_chain CTUs of its slice from the slice-start state, chains spread over threads
 * ========================================================================================== */
#include <pthread.h>
typedef struct {
  const hvxo_hm_pic *P;
  hvxo_hm_ctu_data *ctus;
  int16_t **rec;
  const int *rs;
  const int32_t *chain_first;
  int n_chains, per_chain, slice_ctus, n;
  const uint8_t *entry_states;
  int16_t *out_parts;
  int32_t *out_coef;
  uint8_t *out_recon;
  double *out_cost;
  uint32_t *out_bits_dist;
  int next;
  pthread_mutex_t lock;
} chain_job;

static void chain_run(chain_job *J, int k) {
  const hvxo_hm_pic *P = J->P;
  const int first = J->chain_first[k];
  hvxo_hm_coder cur;
  int16_t int2n[16], next2n[16];
  memset(int2n, 0, sizeof(int2n));
  for (int i = 0; i < J->per_chain; i++) {
    const int a = first + i;
    /* a chain may run over consecutive slices: every slice starts from the slice-start states,
     * m_integerMv2Nx2N carries on (TEncSlice::compressSlice, TEncSearch member state) */
    const int s0 = a - a % J->slice_ctus;
    const int s1 = (s0 + J->slice_ctus < J->n ? s0 + J->slice_ctus : J->n) - 1;
    if (i == 0 || a == s0) {
      memset(&cur, 0, sizeof(cur));
      memcpy(cur.st, J->entry_states, 202);
    }
    hvxo_hm_coder after;
    hvxo_hm_compress_ctu_slice(P, J->ctus, J->rec, J->rs, a, s0, s1, &cur, int2n, next2n, &after);
    cur = after;
    memcpy(int2n, next2n, sizeof(int2n));
    const size_t o = (size_t)k * J->per_chain + i;
    hvxo_hm_ctu_data *q = &J->ctus[a];
    hvxo_hm_unpack_parts(q, J->out_parts + o * 256 * HVXO_HM_PART_FIELDS);
    memcpy(J->out_coef + o * 6144, q->coef[0], sizeof(int32_t) * 4096);
    memcpy(J->out_coef + o * 6144 + 4096, q->coef[1], sizeof(int32_t) * 1024);
    memcpy(J->out_coef + o * 6144 + 5120, q->coef[2], sizeof(int32_t) * 1024);
    J->out_cost[o] = q->cost;
    J->out_bits_dist[2 * o] = q->bits;
    J->out_bits_dist[2 * o + 1] = q->dist;
    const int ax = a % P->w_ctus, ay = a / P->w_ctus;
    uint8_t *r = J->out_recon + o * 6144;
    for (int c = 0; c < 3; c++) {
      const int s = c ? 1 : 0, cs = 64 >> s, W = P->w >> s, H = P->h >> s;
      for (int y = 0; y < cs; y++)
        for (int x = 0; x < cs; x++)
          r[(c ? 4096 + (c - 1) * 1024 : 0) + y * cs + x] =
              (ax * cs + x < W && ay * cs + y < H) ? (uint8_t)J->rec[c][(ay * cs + y) * J->rs[c] + ax * cs + x] : 0;
    }
  }
}
static void *chain_worker(void *arg) {
  chain_job *J = (chain_job *)arg;
  for (;;) {
    pthread_mutex_lock(&J->lock);
    const int k = J->next++;
    pthread_mutex_unlock(&J->lock);
    if (k >= J->n_chains) return NULL;
    chain_run(J, k);
  }
}

int hvxo_hm_chains(const int32_t *pi, const double *pf, const uint8_t *org, const uint8_t *refpics, int n_refpics,
                   const int16_t *col_field, const int32_t *entropy_bits, const uint8_t *entry_states, int n_chains,
                   const int32_t *chain_first, int ctus_per_chain, int slice_ctus, int n_threads, int16_t *out_parts,
                   int32_t *out_coef, uint8_t *out_recon, double *out_cost, uint32_t *out_bits_dist) {
  return hvxo_hm_chains_rd(pi, pf, org, refpics, n_refpics, col_field, entropy_bits, entry_states, n_chains, chain_first,
                           ctus_per_chain, slice_ctus, n_threads, 0, 0.0, out_parts, out_coef, out_recon, out_cost,
                           out_bits_dist);
}
int hvxo_hm_chains_rd(const int32_t *pi, const double *pf, const uint8_t *org, const uint8_t *refpics, int n_refpics,
                      const int16_t *col_field, const int32_t *entropy_bits, const uint8_t *entry_states, int n_chains,
                      const int32_t *chain_first, int ctus_per_chain, int slice_ctus, int n_threads, int rd_metric,
                      double lambda_ssim, int16_t *out_parts, int32_t *out_coef, uint8_t *out_recon, double *out_cost,
                      uint32_t *out_bits_dist) {
  return hvxo_hm_chains_stv(pi, pf, org, refpics, n_refpics, col_field, entropy_bits, entry_states, n_chains, chain_first,
                            ctus_per_chain, slice_ctus, n_threads, rd_metric, lambda_ssim, NULL, out_parts, out_coef,
                            out_recon, out_cost, out_bits_dist);
}
int hvxo_hm_chains_stv(const int32_t *pi, const double *pf, const uint8_t *org, const uint8_t *refpics, int n_refpics,
                       const int16_t *col_field, const int32_t *entropy_bits, const uint8_t *entry_states, int n_chains,
                       const int32_t *chain_first, int ctus_per_chain, int slice_ctus, int n_threads, int rd_metric,
                       double lambda_ssim, const hvxo_stv *stv, int16_t *out_parts, int32_t *out_coef, uint8_t *out_recon,
                       double *out_cost, uint32_t *out_bits_dist) {
  tables_init();
  hvxo_init_tables();
  if (pi[P_COL_VALID] && !col_field) return -1;
  const int w = pi[P_W], h = pi[P_H], wc = (w + 63) / 64, hc = (h + 63) / 64, n = wc * hc;
  for (int k = 0; k < n_chains; k++)
    if (slice_ctus < 1 || ctus_per_chain < 1 || chain_first[k] < 0 || chain_first[k] + ctus_per_chain > n) return -1;
  pic_buf B;
  pic_setup(&B, pi, pf, org, refpics, n_refpics, col_field, entropy_bits);
  B.P.rd_metric = rd_metric;
  B.P.lambda_ssim = lambda_ssim;
  set_stv(&B.P, stv);
  hvxo_hm_ctu_data *ctus = (hvxo_hm_ctu_data *)calloc((size_t)n, sizeof(hvxo_hm_ctu_data));
  const int rw = wc * 64, rh = hc * 64;
  int16_t *recb[3];
  int rs[3] = {rw, rw / 2, rw / 2};
  for (int c = 0; c < 3; c++) recb[c] = (int16_t *)calloc((size_t)(c ? rw * rh / 4 : rw * rh), sizeof(int16_t));
  chain_job J;
  memset(&J, 0, sizeof(J));
  J.P = &B.P; J.ctus = ctus; J.rec = recb; J.rs = rs; J.chain_first = chain_first;
  J.n_chains = n_chains; J.per_chain = ctus_per_chain; J.slice_ctus = slice_ctus; J.n = n;
  J.entry_states = entry_states; J.out_parts = out_parts; J.out_coef = out_coef; J.out_recon = out_recon;
  J.out_cost = out_cost; J.out_bits_dist = out_bits_dist;
  pthread_mutex_init(&J.lock, NULL);
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 64) n_threads = 64;
  pthread_t th[64];
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, chain_worker, &J);
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&J.lock);
  for (int c = 0; c < 3; c++) free(recb[c]);
  pic_free(&B);
  free(ctus);
  return n_chains * ctus_per_chain;
}

void hvxo_hm_unpack_parts(const hvxo_hm_ctu_data *d, int16_t *out /* [256][HVXO_HM_PART_FIELDS] */) {
  for (int z = 0; z < 256; z++) {
    const hm_part *p = &d->p[z];
    int16_t *u = out + z * HVXO_HM_PART_FIELDS;
    u[0] = p->depth; u[1] = p->part; u[2] = p->pred; u[3] = p->skip; u[4] = p->merge; u[5] = p->merge_idx;
    u[6] = p->inter_dir; u[7] = p->ref[0]; u[8] = p->ref[1];
    u[9] = p->mv[0][0]; u[10] = p->mv[0][1]; u[11] = p->mv[1][0]; u[12] = p->mv[1][1];
    u[13] = p->mvd[0][0]; u[14] = p->mvd[0][1]; u[15] = p->mvd[1][0]; u[16] = p->mvd[1][1];
    u[17] = p->mvp_idx[0]; u[18] = p->mvp_idx[1]; u[19] = p->idir[0]; u[20] = p->idir[1]; u[21] = p->tr_idx;
    u[22] = p->ts[0]; u[23] = p->ts[1]; u[24] = p->ts[2]; u[25] = p->cbf[0]; u[26] = p->cbf[1]; u[27] = p->cbf[2];
    u[28] = p->qp;
  }
}
void hvxo_hm_pack_parts(hvxo_hm_ctu_data *d, const int16_t *in) {
  for (int z = 0; z < 256; z++) {
    hm_part *p = &d->p[z];
    const int16_t *u = in + z * HVXO_HM_PART_FIELDS;
    memset(p, 0, sizeof(*p));
    p->depth = (int8_t)u[0]; p->part = (int8_t)u[1]; p->pred = (int8_t)u[2]; p->skip = (int8_t)u[3];
    p->merge = (int8_t)u[4]; p->merge_idx = (int8_t)u[5]; p->inter_dir = (int8_t)u[6];
    p->ref[0] = (int8_t)u[7]; p->ref[1] = (int8_t)u[8];
    p->mv[0][0] = u[9]; p->mv[0][1] = u[10]; p->mv[1][0] = u[11]; p->mv[1][1] = u[12];
    p->mvd[0][0] = u[13]; p->mvd[0][1] = u[14]; p->mvd[1][0] = u[15]; p->mvd[1][1] = u[16];
    p->mvp_idx[0] = (int8_t)u[17]; p->mvp_idx[1] = (int8_t)u[18];
    p->idir[0] = (uint8_t)u[19]; p->idir[1] = (uint8_t)u[20]; p->tr_idx = (int8_t)u[21];
    p->ts[0] = (uint8_t)u[22]; p->ts[1] = (uint8_t)u[23]; p->ts[2] = (uint8_t)u[24];
    p->cbf[0] = (uint8_t)u[25]; p->cbf[1] = (uint8_t)u[26]; p->cbf[2] = (uint8_t)u[27];
    p->qp = (int8_t)u[28];
    p->width = (uint8_t)(64 >> p->depth);
  }
}
size_t hvxo_hm_ctu_data_size(void) { return sizeof(hvxo_hm_ctu_data); }

void hvxo_hm_derive_lists(hvxo_hm_pic *P) {
  const int isb = P->slice_type == B_SLICE;
  int gpb = isb && P->nref[0] == P->nref[1];
  for (int i = 0; gpb && i < P->nref[1]; i++)
    if (P->ref_poc[1][i] != P->ref_poc[0][i]) gpb = 0;
  P->mvd_l1_zero = gpb;
  for (int i = 0; i < 4; i++) {
    P->l1_to_l0[i] = -1;
    if (!isb || i >= P->nref[1]) continue;
    for (int k = 0; k < P->nref[0]; k++)
      if (P->ref_poc[0][k] == P->ref_poc[1][i]) { P->l1_to_l0[i] = k; break; }
  }
}

/* ============================================================================================
 * Loop filter inputs and compressed motion of a decided picture (hvx_oracle_cu.h)
 * ========================================================================================== */
enum { PF_DEPTH = 0, PF_PART = 1, PF_PRED = 2, PF_REF0 = 7, PF_REF1 = 8, PF_MV0X = 9, PF_TR_IDX = 21, PF_CBF_Y = 25,
       PF_QP = 28 };

/* the z-order index of the 4x4 unit (ux, uy) of a CTU (g_auiRasterToZscan: x bits interleaved below y bits) */
static int unit_z(int ux, int uy) {
  int z = 0;
  for (int b = 0; b < 4; b++) z |= (((ux >> b) & 1) << (2 * b)) | (((uy >> b) & 1) << (2 * b + 1));
  return z;
}
static const int16_t *unit_part(const int16_t *parts, int wc, int x, int y) {
  const int a = (y >> 6) * wc + (x >> 6);
  return parts + ((size_t)a * 256 + unit_z((x & 63) >> 2, (y & 63) >> 2)) * HVXO_HM_PART_FIELDS;
}
/* the unit's reference picture of list l (TComSlice::getRefPic), by POC; INT32_MIN = none (NULL) */
static int32_t unit_ref(const int16_t *q, const int32_t *ref_poc, int l) {
  const int r = q[PF_REF0 + l];
  return r < 0 ? INT32_MIN : ref_poc[l * 4 + r];
}
static int mv_far(const int *a, const int *b) { return abs(a[0] - b[0]) >= 4 || abs(a[1] - b[1]) >= 4; }

/* one unit's edge in direction dir (0 vertical / left, 1 horizontal / top) at luma (x, y) */
static int unit_bs(const int16_t *parts, int wc, int x, int y, int dir, const int32_t *ref_poc, int is_b) {
  if (dir == 0 ? (x & 7) : (y & 7)) return 0;  /* only the 8x8 grid is read (xEdgeFilterLuma's iEdge step, :220) */
  if (dir == 0 ? x == 0 : y == 0) return 0;    /* picture border: bLeftEdge / bTopEdge false (:372, :394) */
  const int16_t *q = unit_part(parts, wc, x, y);
  const int cs = 64 >> q[PF_DEPTH];
  const int r = dir == 0 ? (x & 63) % cs : (y & 63) % cs;  /* position inside the CU along the edge normal */
  /* xSetEdgefilterTU: every TU's left / top edge (the CU's own included, then kept by
   * xSetEdgefilterPU's bLeftEdge / bTopEdge, true inside the picture with LFCrossSliceBoundaryFlag);
   * these edges also carry the "transform edge" mark m_aapucBS tests against the cbfs */
  const int tsz = cs >> q[PF_TR_IDX];
  const int tu_edge = r % tsz == 0;
  /* xSetEdgefilterPU: the internal PU edges of the partition (no transform mark) */
  int pu_edge = 0;
  switch (q[PF_PART]) {
    case 1: pu_edge = dir == 1 && r == cs / 2; break;            /* SIZE_2NxN */
    case 2: pu_edge = dir == 0 && r == cs / 2; break;            /* SIZE_Nx2N */
    case 3: pu_edge = r == cs / 2; break;                        /* SIZE_NxN */
    case 4: pu_edge = dir == 1 && r == cs / 4; break;            /* SIZE_2NxnU */
    case 5: pu_edge = dir == 1 && r == cs - cs / 4; break;       /* SIZE_2NxnD */
    case 6: pu_edge = dir == 0 && r == cs / 4; break;            /* SIZE_nLx2N */
    case 7: pu_edge = dir == 0 && r == cs - cs / 4; break;       /* SIZE_nRx2N */
    default: break;
  }
  if (!tu_edge && !pu_edge) return 0;
  /* xGetBoundaryStrengthSingle (:417) */
  const int16_t *p = dir == 0 ? unit_part(parts, wc, x - 4, y) : unit_part(parts, wc, x, y - 4);
  if (p[PF_PRED] == 1 || q[PF_PRED] == 1) return 2;  /* MODE_INTRA */
  const int cbf_q = (q[PF_CBF_Y] >> q[PF_TR_IDX]) & 1, cbf_p = (p[PF_CBF_Y] >> p[PF_TR_IDX]) & 1;
  if (tu_edge && (cbf_q || cbf_p)) return 1;
  int mp[2][2], mq[2][2];
  int32_t rp[2], rq[2];
  for (int l = 0; l < 2; l++) {
    rp[l] = unit_ref(p, ref_poc, l);
    rq[l] = unit_ref(q, ref_poc, l);
    for (int c = 0; c < 2; c++) {
      mp[l][c] = rp[l] == INT32_MIN ? 0 : p[PF_MV0X + 2 * l + c];
      mq[l][c] = rq[l] == INT32_MIN ? 0 : q[PF_MV0X + 2 * l + c];
    }
  }
  if (!is_b) return (rp[0] != rq[0] || mv_far(mq[0], mp[0])) ? 1 : 0;
  if ((rp[0] == rq[0] && rp[1] == rq[1]) || (rp[0] == rq[1] && rp[1] == rq[0])) {
    if (rp[0] != rp[1]) {
      if (rp[0] == rq[0]) return (mv_far(mq[0], mp[0]) || mv_far(mq[1], mp[1])) ? 1 : 0;
      return (mv_far(mq[1], mp[0]) || mv_far(mq[0], mp[1])) ? 1 : 0;
    }
    return ((mv_far(mq[0], mp[0]) || mv_far(mq[1], mp[1])) && (mv_far(mq[1], mp[0]) || mv_far(mq[0], mp[1]))) ? 1 : 0;
  }
  return 1;
}

void hvxo_hm_boundary_strength(int w, int h, const int16_t *hm_parts, const int32_t *ref_poc, int is_b,
                               uint8_t *bs_ver, uint8_t *bs_hor, int8_t *qp) {
  const int wc = (w + 63) / 64, uw = w / 4, uh = h / 4;
  for (int uy = 0; uy < uh; uy++)
    for (int ux = 0; ux < uw; ux++) {
      const int x = ux * 4, y = uy * 4, i = uy * uw + ux;
      bs_ver[i] = (uint8_t)unit_bs(hm_parts, wc, x, y, 0, ref_poc, is_b);
      bs_hor[i] = (uint8_t)unit_bs(hm_parts, wc, x, y, 1, ref_poc, is_b);
      qp[i] = (int8_t)unit_part(hm_parts, wc, x, y)[PF_QP];
    }
}

void hvxo_hm_col_field(int w, int h, const int16_t *hm_parts, int16_t *col_field) {
  const int wc = (w + 63) / 64, hc = (h + 63) / 64;
  for (int a = 0; a < wc * hc; a++)
    for (int b = 0; b < 16; b++) {  /* the 16x16 blocks in z-order (parts 0, 16, 32, ...) */
      const int bx = (b & 1) | ((b >> 1) & 2), by = ((b >> 1) & 1) | ((b >> 2) & 2);
      const int x = (a % wc) * 64 + bx * 16, y = (a / wc) * 64 + by * 16;
      const int16_t *q = hm_parts + ((size_t)a * 256 + b * 16) * HVXO_HM_PART_FIELDS;
      int16_t *o = col_field + ((size_t)a * 16 + b) * 8;
      o[0] = (x >= w || y >= h) ? -1 : q[PF_PRED];  /* NUMBER_OF_PART_SIZES outside the picture */
      o[1] = q[PF_REF0];
      o[2] = q[PF_REF1];
      for (int k = 0; k < 4; k++) o[3 + k] = q[PF_MV0X + k];
      o[7] = 0;
    }
}

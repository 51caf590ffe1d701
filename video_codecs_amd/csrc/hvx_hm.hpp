// hvx_hm.hpp -- the HM-exact CTU decision on the device (gfx950): TEncCu::compressCtu
// (TEncCu.cpp:228) with the CTU syntax walk TEncCu::encodeCtu (:252) that carries the CABAC
// contexts from CTU to CTU (TEncSlice.cpp:814-828).
//
// Mapping: ONE 64-lane wave (one workgroup) per chain of CTUs.  HM's decision is a deep,
// data-dependent control flow (xCompressCU recursion, merge/AMVP candidate lists, RQT and
// intra TU recursions, every decision reading the CABAC states the previous one left), so a
// chain is walked in HM's exact order by the whole wave: the control flow is wave-uniform
// (every lane executes it with the same values), and every data-parallel leaf is spread over
// the 64 lanes -- motion search (TZ integer + fractional, hvx_me.hpp), motion compensation,
// forward transform / RDOQ / inverse (hvx_tu.hpp), SSE / SATD / SAD, intra reference samples
// and predictions, the 35-mode first pass, sample copies.  Throughput comes from many
// independent chains (slices, segments, pictures) in flight, one wave each.
//
// Memory: the small, hot state lives in LDS (hm_e: the picture descriptor, the 37 RD coders
// of m_pppcRDSbacCoder + the go-on coder, estBits, the CABAC tables, the leaf scratch union);
// the CU objects (TComDataCU per depth, best/temp), the TComYuv buffers and the QT temporaries
// live in a per-chain State in HBM.  The CTU being decided keeps its TComPic data and its
// reconstruction in the State too (cur CTU window), so that chains never write what another
// chain reads while it runs; a chained job publishes each finished CTU into the picture.
//
// Each function below restates the oracle function of the same name in
// oracle/hvx_oracle_cu.c (which cites the HM function it follows) and is pinned, like the
// oracle, against the reference's own compressCtu decisions (tests/golden/ctu_ldp_*.bin).
#pragma once
#include "hvx_dev.hpp"
#ifdef HM_PROFILE
__device__ void hm_prof_add(int cat, uint64_t dt);
#define HVX_TU_PROF_HOOK(cat, dt) hm_prof_add((cat), (dt))
#endif
#include "hvx_tu.hpp"
#include "hvx_cabac.hpp"
#include "hvx_estbit.hpp"
#include "hvx_mc.hpp"
#include "hvx_intra.hpp"
#include "hvx_me.hpp"
#include "hvx_ssimw.hpp"

namespace hm {

constexpr double kMaxDouble = 1.7e+308;
constexpr uint32_t kMaxU32 = 0xffffffffu;
enum { SIZE_2Nx2N, SIZE_2NxN, SIZE_Nx2N, SIZE_NxN, SIZE_2NxnU, SIZE_2NxnD, SIZE_nLx2N, SIZE_nRx2N, SIZE_NONE };
enum { MODE_INTER = 0, MODE_INTRA = 1, MODE_NONE = 2 };
enum { CI_CURR_BEST, CI_NEXT_BEST, CI_TEMP_BEST, CI_CHROMA_INTRA, CI_QT_TRAFO_TEST, CI_QT_TRAFO_ROOT, CI_NUM };
enum { B_SLICE = 0, P_SLICE = 1, I_SLICE = 2 };
constexpr int DM_CHROMA_IDX = 36;
// context offsets in TEncSbac::m_contextModels (TEncSbac.cpp:62-92)
enum {
  X_SPLIT = 0, X_SKIP = 3, X_MERGE_FLAG = 6, X_MERGE_IDX = 7, X_PART = 8, X_PRED = 12, X_INTRA = 13, X_CHROMA = 14,
  X_INTER_DIR = 19, X_REF = 24, X_MVD = 26, X_QT_CBF = 28, X_SUBDIV = 38, X_ROOT_CBF = 41, X_MVP = 180,
  X_SAO_MERGE = 181, X_SAO_TYPE = 182
};
constexpr int GOON = 36;  // m_pcRDGoOnSbacCoder; rd coders are d * 6 + ci
__device__ __forceinline__ int RD(int d, int ci) { return d * CI_NUM + ci; }

typedef hvx_hm_part Part;
typedef hvx_hm_coder Coder;

// z-order <-> raster of the 16x16 partition grid (g_auiZscanToRaster, TComRom.cpp:196-260)
__device__ __forceinline__ int z2r(int z) {
  const int x = (z & 1) | ((z >> 1) & 2) | ((z >> 2) & 4) | ((z >> 3) & 8);
  const int y = ((z >> 1) & 1) | ((z >> 2) & 2) | ((z >> 3) & 4) | ((z >> 4) & 8);
  return y * 16 + x;
}
__device__ __forceinline__ int r2z(int r) {
  const int x = r & 15, y = r >> 4;
  return (x & 1) | ((y & 1) << 1) | ((x & 2) << 1) | ((y & 2) << 2) | ((x & 4) << 2) | ((y & 4) << 3) | ((x & 8) << 3) |
         ((y & 8) << 4);
}
__device__ __forceinline__ int rpx(int r) { return (r & 15) << 2; }
__device__ __forceinline__ int rpy(int r) { return (r >> 4) << 2; }
__device__ __forceinline__ int ilog2(int n) { return 31 - __builtin_clz(n); }

// a CU object of TEncCu (m_ppcBestCU / m_ppcTempCU of one depth)
struct Cu {
  int depth, zidx, x, y, nparts, width;
  uint32_t bits, dist;
  double cost;
  double dssim;  // HVX_RD_SSIM: the SSIM distortion of the CU's reconstruction (cu_dssim)
  int merge_amp, pad_;
  Part p[256];
  int16_t coef[6144];  // Y 4096 | Cb 1024 | Cr 1024, TU-packed
};
__device__ __forceinline__ int coff(int c) { return c == 0 ? 0 : c == 1 ? 4096 : 5120; }

// a TComYuv of a CU up to 64x64, packed for the CU being decided (width W = Enc.yw): Y W x W
// (stride W) | Cb | Cr (W/2 x W/2, stride W/2).  An 8x8 CU's buffer is 192 contiguous bytes (two
// cache lines) instead of a 64-stride 64x64 layout's sixteen.
struct Yuv { int16_t s[6144]; };

// the leaf scratch of motion search and motion compensation (in the chain state: global memory)
struct MeScratch {
  union {
    MeFracSmem<64, 1> sm;             // uni search: the original (8-bit) pattern
    MeFracSmem<64, 1, int16_t> sm16;  // bi refinement: the 2 * org - pred(other list) target
  };
  uint32_t red[2 * kMeMaxRanges];
  hvx_me_result r;
};
struct McScratch {
  int16_t tmp[(64 + 7) * 64];
  int16_t pr[2][64 * 64];
};
struct IntraScratch {
  int16_t unf[intra::kB + 3], filt[intra::kB + 3];
  uint8_t org[64 * 64];
  uint32_t satd[36];
  int list[12], mpm[3];
  double cc[10];
  int n_cand, pad_;
  uint8_t cand[12];
};
// A codeCoeffNxN count of a 4x4 / 8x8 TU, remembered: its result (the bits it added, the context
// states it left) is a function of the TU's levels, its descriptor fields the walk reads (width,
// channel, scan, transform skip) and the states of the channel's coefficient contexts before the
// count.  The RQT counts the same TU from the same states several times (the per-component test
// from CI_QT_TRAFO_ROOT, the node's single-bits recount, the parent's split recount, the CU's
// final count), so a chain keeps its last kMemoK counts (FIFO) and replays a repeated one.
// Context rows 40..187 as 37 dwords; a per-channel byte mask selects the rows the walk touches.
#ifndef HM_MEMO_K
#define HM_MEMO_K 64
#endif
#ifndef HM_MEMO_B
#define HM_MEMO_B 16
#endif
constexpr int kMemoK = HM_MEMO_K, kMemoDw = 37, kMemoDw0 = 10;
struct CoefMemo {
  uint32_t key;                   // valid | width | channel | scan | transform skip
  uint32_t hash;                  // memo_hash of the entry's levels and masked context states
  uint64_t frac;
  uint32_t coef[32];              // the TU's levels as int16 pairs (TU-packed order)
  uint32_t before[kMemoDw], after[kMemoDw];
};
// 16x16 / 32x32 counts (HM_MEMO_BIG): a short FIFO of their own -- the RQT counts a TU once while
// choosing its mode and again for the node's total (the coefficient contexts unchanged between)
constexpr int kMemoB = HM_MEMO_B;
struct CoefMemoBig {
  uint32_t key, hash;
  uint64_t frac;
  uint32_t before[kMemoDw], after[kMemoDw];
  uint32_t coef[512];             // int16 pairs (TU-packed order); dword k * 64 + lane
};
// The inter residual memo (enc_res_rd_inter): xEstimateInterResidualQT and the residual decision
// after it depend only on the CU's residual and the RD coder they start from
// (m_pppcRDSbacCoder[depth][CI_CURR_BEST]); within one CU the residual is fixed by the PUs' motion
// (the merge candidates, the 2Nx2N search and the merge candidates of the other partitions repeat
// motion: ~30% of the inter RQTs on the LDP / RA captures).  An entry per CU depth holds the first
// kRqK distinct (partition, motion, start coder) keys of the CU being decided and what the RQT left
// that is read afterwards: every partition's tr_idx / transform-skip / cbf bytes, the CU's
// coefficients (unless the residual was dropped) and resi_best.  Entry layout: header (64 dwords:
// the start coder's 54 dwords, 6 key dwords, the "dropped" flag) | 8 B per partition | coefficients
// Y | Cb | Cr (1.5 W^2 int16) | resi_best (1.5 W^2 int16, the packed TComYuv).  Two entries catch
// 99% of the repeats (the restatement's count on the captures).  The helpers stay out of line: inlined
// they change how enc_res_rd_inter inlines the RQT root, and that build ran 2.3% slower.
constexpr int kRqK = 2;
__host__ __device__ constexpr int rq_entry_bytes(int d) {
  return 256 + 8 * (256 >> (2 * d)) + 2 * 3 * (64 >> d) * (64 >> d);
}
__host__ __device__ constexpr int rq_depth_off(int d) {
  return d == 0 ? 0 : rq_depth_off(d - 1) + kRqK * rq_entry_bytes(d - 1);
}
constexpr int kRqBytes = rq_depth_off(4);
// per-chain state in HBM
struct State {
  int status[4];  // [0]: the job's status word (hvx_hm_job_status: 0 ran, -HVX_HM_BAD_* refused)
  int dbg[4];     // HM_CHECKS: E.dbg of the last CTU
  uint64_t prof[2][32];  // HM_PROFILE: per-category clock ticks and calls of the job
  Cu cu[8];
  Yuv yuv[28];                    // TComYuv sets (kind x depth), addressed through hm_e.yi
  Yuv qt_yuv[4], qt_ts_yuv, tmp_yuv_pred;
  int16_t pred_l[2][64 * 64];     // TEncSearch::m_acYuvPred[list] (luma: the bi search's other-list prediction)
  int16_t qt_coef[4][6144];       // m_ppcQTTempCoeff[comp][layer]
  int16_t qt_tu_coef[6144];       // m_pcQTTempTUCoeff (Y | Cb | Cr)
  int16_t shared_pred[6144];      // m_pSharedPredTransformSkip
  int16_t rq_best_coef[4][1024], rq_best_res[4][1024];
  uint8_t tmp_tridx[256], tmp_cbf[3][256], tmp_ts[3][256];
  uint8_t save_cbf[3][256], save_ts[3][256];
  Cu view;                        // encodeCtu's CU-relative view of the CTU
  Part ctu_p[256];                // TComPic::getCtu(addr) of the CTU being decided
  int16_t ctu_coef[6144];
  uint32_t ctu_bits, ctu_dist;
  double ctu_cost;
  uint8_t win[6144];              // its reconstruction: Y 64x64 | Cb 32x32 | Cr 32x32
  int16_t int2n[2][4][2];         // TEncSearch::m_integerMv2Nx2N
  Coder carry;                    // the RD coder after the chain's last encodeCtu (HVX_HM_RESUME)
  CoefMemo memo[kMemoK];          // codeCoeffNxN counts of 4x4 / 8x8 TUs the chain made recently
  int memo_next;
  CoefMemoBig memob[kMemoB];      // ... and of 16x16 / 32x32 TUs
  int memob_next;
  alignas(16) uint8_t rq_data[kRqBytes];  // the inter residual memo's entries (per CU depth)
  int rq_n[4];                            // ... entries held for the CU being decided at each depth
  MeScratch me;                   // leaf scratch outside LDS
  McScratch mc;
  TuSmem<3> tu3;
};

// the LDS leaf scratch (one leaf runs at a time): TU pipelines up to 16x16 and the intra
// first pass.  The 32x32 TU pipeline, motion search and motion compensation keep theirs in the
// chain state (global memory), which holds the LDS footprint of a chain's wave under 20 KB (8 waves per CU)
union Leaf {
  TuSmem<0> tu0;
  TuSmem<1> tu1;
  TuSmem<2> tu2;
  IntraScratch in;
  struct {               // codeCoeffNxN's TU staged in scan order (code_coeff_nxn)
    int16_t lev[1024];   // levels
    int16_t ras[256];    // raster position (TUs up to 16x16)
    int32_t sig[256];    // significance context under neighbour-CG patterns 0..3, 6 bits each
    uint8_t cg[64];      // CG scan -> CG raster
  } cs;
};

// a TComTU / TComTURecurse node (4:2:0 rectangles relative to the CU).  The nodes live on a stack
// in LDS (Enc.tstack, TuSlot): wave-uniform, and a per-lane copy lived in scratch (call-frame
// traffic on every field read through a reference)
struct Tu {
  int cu_depth, cu_zidx;
  int split, section, last_of_level;
  int rel, step, log2;
  int trd[3], x0[3], y0[3], w[3], h[3], ow[3], all[3], off[3];
};
constexpr int kTuStack = 10;

// AMVP candidates of one (list, reference) (AMVPInfo)
struct Amvp { int n; int16_t c[3][2]; };
// predInterSearch's per-PU records (TEncSearch.cpp:2937-2995: cMvTemp, cMvPred(Bi), aaiMvpIdx(Bi),
// aaiMvpNum, aacAMVPInfo, uiCostTempL0, ...): wave-uniform, indexed by list / reference, in LDS
struct InterSearch {
  Amvp amvp[2][4];
  int16_t mvtemp[2][4][2], mvpred[2][4][2], mvpredbi[2][4][2];
  int mvp_idx[2][4], mvp_num[2][4], mvp_idx_bi[2][4];
  uint32_t cost_l0[4], bits_l0[4];
  uint32_t cost[2], bits[3], motbits[2];
  int16_t mv[2][2], mvbi[2][2];
  int ref[2], refbi[2];
};

// the decision's LDS-resident context (TEncCu / TEncSearch / TComTrQuant scalars + coders)
struct Enc {
  hvx_hm_picture P;
  State *S;
  int ctu_addr, ctu_x, ctu_y, slice_qp;
  int slice_start, slice_end;  // the chain's slice (CTU addresses)
  int best[4], temp[4];  // Cu index in S->cu
  int yi[7][4];          // Yuv index: orig, pred_best, pred_temp, resi_best, resi_temp, reco_best, reco_temp
  int cur;               // the coder the entropy calls count with
  int pad_;
  Coder cod[37];
  hvx_estbits est;
  uint32_t est_key;      // (w | h << 8 | ch << 16) + 1 of the last estimate_bit (0: none this CTU)
  uint32_t est_st[38];   // its coder's context states 28 .. 179 (every byte estBit reads)
  // one LDS word per (CABAC state q, bin v), entry 2q + v: the next state (ContextModel::update) in
  // bits 24..31, ContextModel::m_entropyBits[q ^ v] in bits 0..23 -- a counted bin is one LDS read
  uint32_t pk[256];
  uint16_t scan[256];    // the current TU's scan tables (TUs up to 16x16), staged by tu_fwd_l
  uint8_t scan_cg[16];
  uint32_t avail[4];
  InterSearch is;
  hvx_tu_desc td;        // the current TU's descriptor (tu_desc)
  Tu tstack[kTuStack];   // the live TU nodes (TuSlot), innermost last
  int tsp;
  uint32_t memo_key[kMemoK], memo_hash[kMemoK];  // the count memo's index (S->memo keys / hashes)
  int memo_next;
  uint32_t memob_key[kMemoB], memob_hash[kMemoB];
  int memob_next;
  int yw;                // the width of the CU whose TComYuv buffers are in use (compress_cu<D>: 64 >> D)
  float ssim_t[192];     // HVX_RD_SSIM: the (1 - SSIM) terms of a CU's blocks (cu_dssim)
  int dbg[4];  // HM_CHECKS: first violated check (code, a, b) of the job
  int stage, stop;  // HM_CHECKS: stop the CTU at debugging stage `stage` (0: never)
#ifdef HM_PROFILE
  uint64_t prof[2][32];  // HM_PROFILE accumulators
#endif
  Leaf u;
};
}  // namespace hm

__shared__ hm::Enc hm_e;

// Enc.pk from ContextModel::m_entropyBits (eb: 128 int32, or nullptr: zeros) and the state
// transitions of ContextModel::updateMPS / updateLPS; lane l fills entries l, l + 64, l + 128, l + 192
__device__ __forceinline__ void hm_fill_pk(const int32_t *eb, int l) {
  for (int j = l; j < 256; j += 64) {
    const int q = j >> 1, v = j & 1, p = q >> 1, mps = q & 1;
    const int ns = v == mps ? (((p < 62 ? p + 1 : p) << 1) | mps) : ((cab::kTransIdxLps[p] << 1) | (p == 0 ? mps ^ 1 : mps));
    hm_e.pk[j] = ((uint32_t)ns << 24) | ((eb ? (uint32_t)eb[q ^ v] : 0u) & 0xffffffu);
  }
}

#ifdef HM_PROFILE
// s_memtime is the shader clock of the XCD the wave runs on: a wave that the driver preempts and
// restores elsewhere can read an earlier time at the end of a scope than at its start.  Such an
// interval counts as 0 ticks (it was what wrapped the round-5 accumulators to ~1.8e19).
__device__ __forceinline__ uint64_t hm_prof_dt(uint64_t t0, uint64_t t1) { return (int64_t)(t1 - t0) > 0 ? t1 - t0 : 0; }
__device__ void hm_prof_add(int cat, uint64_t dt) {
  hm_e.prof[0][cat] += (int64_t)dt > 0 ? dt : 0;
  hm_e.prof[1][cat] += 1;
}
#endif

namespace hm {
#define E hm_e
// the packed table's two halves (Enc.pk)
__device__ __forceinline__ uint32_t ebits(int x) { return E.pk[2 * x] & 0xffffffu; }
__device__ __forceinline__ int nstate(int j) { return (int)(E.pk[j] >> 24); }
enum { Y_ORIG, Y_PRED_BEST, Y_PRED_TEMP, Y_RESI_BEST, Y_RESI_TEMP, Y_RECO_BEST, Y_RECO_TEMP };
__device__ __forceinline__ Yuv *YB(int kind, int d) { return &E.S->yuv[E.yi[kind][d]]; }
__device__ __forceinline__ Cu *BEST(int d) { return &E.S->cu[E.best[d]]; }
__device__ __forceinline__ Cu *TEMP(int d) { return &E.S->cu[E.temp[d]]; }
// a chain is one wave (its workgroup): the compiler already lowers this to wavefront-scope
// ordering (no s_barrier, no wait for outstanding stores; checked in the ISA)
__device__ __forceinline__ void wsync() { __syncthreads(); }
__device__ __forceinline__ int lid() { return (int)threadIdx.x; }
// the TComYuv layout of the CU being decided (E.yw)
__device__ __forceinline__ int ystride(int c) { return c ? E.yw >> 1 : E.yw; }
__device__ __forceinline__ int ycoff(int c, int w) { return c == 0 ? 0 : c == 1 ? w * w : w * w + (w * w >> 2); }
__device__ __forceinline__ int16_t *yaddr_w(Yuv *b, int c, int x, int y, int w) {
  return b->s + ycoff(c, w) + y * (c ? w >> 1 : w) + x;
}
__device__ __forceinline__ int16_t *yaddr(Yuv *b, int c, int x, int y) { return yaddr_w(b, c, x, y, E.yw); }
// HM_PROFILE builds accumulate the clock ticks (s_memtime) and calls of the leaf categories
enum { PR_ME, PR_MC, PR_TPL, PR_TUF, PR_TUI, PR_COEF, PR_EST, PR_IFP, PR_IPRED, PR_DIST, PR_CTU, PR_ENC, PR_N };
// sub-phases (HM_PROFILE): 12..15 TUF by size; 16 COEF descriptor, 17 COEF staging, 18 COEF walk,
// 19 TUF copy-in, 20 TUF forward (transform + quantisation), 21 TUF copy-out, 22 transform,
// 23 RDOQ, 24..27 COEF by size
enum { PR_COEF_DESC = 16, PR_COEF_STAGE, PR_COEF_WALK, PR_TUF_IN, PR_TUF_FWD, PR_TUF_OUT, PR_XFORM, PR_RDOQ, PR_COEF4 };
#ifdef HM_PROFILE
struct ProfScope {
  int cat;
  uint64_t t0;
  __device__ __forceinline__ explicit ProfScope(int c) : cat(c), t0(__builtin_amdgcn_s_memtime()) {}
  __device__ __forceinline__ ~ProfScope() {
    hm_e.prof[0][cat] += hm_prof_dt(t0, __builtin_amdgcn_s_memtime());
    hm_e.prof[1][cat] += 1;
  }
};
#define HM_PROF(c) ProfScope prof_scope_(c)
#define HM_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define HM_TADD(cat, v) (hm_e.prof[0][(cat)] += hm_prof_dt((v), __builtin_amdgcn_s_memtime()), hm_e.prof[1][(cat)] += 1)
#else
#define HM_T0(v) ((void)0)
#define HM_TADD(cat, v) ((void)0)
#define HM_PROF(c) ((void)0)
#endif
#ifndef HM_WT0
#define HM_WT0(v) ((void)0)
#define HM_WTADD(k, v) ((void)0)
#endif
// HM_CHECKS builds validate the indices and sample positions below, record the first violation
// in E.dbg and keep the access inside its buffer (a debugging aid; off in the product build)
#ifdef HM_CHECKS
__device__ __noinline__ void hm_fail(int code, int a, int b) {
  if (E.dbg[0] == 0) { E.dbg[0] = code; E.dbg[1] = a; E.dbg[2] = b; }
}
#define HMC(cond, code, a, b) do { if (!(cond)) hm_fail((code), (a), (b)); } while (0)
#define HM_CHECKING 1
#define HM_STAGE(k) do { if (E.stage == (k)) E.stop = 1; } while (0)
#define HM_STOPPED (E.stop)
#else
#define HMC(cond, code, a, b) ((void)0)
#define HM_CHECKING 0
#define HM_STAGE(k) ((void)0)
#define HM_STOPPED 0
#endif

// a TU node on the LDS stack for the scope of the object (declared like a local: TU_LOCAL(ch))
// (the deepest nesting is 6 nodes: est_intra_pred_luma_qt's CU and PU nodes + four RQT levels, or
// an RQT level's children + encode_inter_residual_qt's descent; HM_CHECKS builds bound it)
__device__ __forceinline__ int tu_push() {
  const int k = E.tsp;
  HMC(k >= 0 && k < kTuStack, 90, k, 0);
  E.tsp = k + 1;
  return HM_CHECKING ? (k < 0 ? 0 : k >= kTuStack ? kTuStack - 1 : k) : k;
}
struct TuSlot {
  Tu &t;
  __device__ __forceinline__ TuSlot() : t(E.tstack[tu_push()]) {}
  __device__ __forceinline__ ~TuSlot() { E.tsp = E.tsp - 1; }
};
#define TU_LOCAL(name) TuSlot name##_slot_; Tu &name = name##_slot_.t

// ============================================================================================
// CABAC bit counter over the coders in LDS (cbin/cep/ctrm/reset_bits/written_bits/load)
// ============================================================================================
__device__ __forceinline__ void cbin(int ctx, int v) {
  Coder &c = E.cod[E.cur];
  const int s = c.st[ctx];
  const uint32_t pv = E.pk[s * 2 + v];
  c.frac += pv & 0xffffffu;
  c.st[ctx] = (uint8_t)(pv >> 24);
}
__device__ __forceinline__ void cep(int n) { E.cod[E.cur].frac += 32768ull * (uint32_t)n; }
__device__ __forceinline__ void ctrm(int v) { E.cod[E.cur].frac += ebits(126 ^ v); }
__device__ __forceinline__ void reset_bits() { E.cod[E.cur].frac &= 32767; }
__device__ __forceinline__ uint32_t written_bits() { return (uint32_t)(E.cod[E.cur].frac >> 15); }
__device__ __forceinline__ void cload(int dst, int src) {
  HMC(dst >= 0 && dst < 37 && src >= 0 && src < 37, 8, dst, src);
  uint32_t *d = (uint32_t *)&E.cod[dst];
  const uint32_t *s = (const uint32_t *)&E.cod[src];
  const int l = lid();
  uint32_t v = l < 54 ? s[l] : 0;
  wsync();
  if (l < 54) d[l] = v;
  wsync();
}

// a wave-uniform value read from LDS (a marker: moving these to scalar registers with readfirstlane
// was measured 7% slower -- the round trips lengthen the dependent chains)
__device__ __forceinline__ int uni(int v) { return v; }

// the coefficient-rate lane of cab::coeff_bits on one coder (models 42..184)
struct CoderLane {
  uint8_t *st;
  uint64_t frac;
  __device__ __forceinline__ void bin(int row, int v) {
    uint8_t &s = st[uni(row) + cab::kCtxLo];
    const int q = uni(s), bv = uni(v);
    const uint32_t pv = (uint32_t)uni((int)E.pk[q * 2 + bv]);
    frac += pv & 0xffffffu;
    s = (uint8_t)(pv >> 24);
  }
  __device__ __forceinline__ void ep(int n) { frac += 32768ull * (uint32_t)n; }
  __device__ __forceinline__ void ep_bits(uint32_t, int n) { ep(n); }
  __device__ __forceinline__ void eps(uint32_t, int n) { ep(n); }
  __device__ __forceinline__ void esc(uint32_t symbol, int r, bool limited, int max_log2) {
    ep(cab::remain_bins(symbol, r, limited, max_log2));
  }
};

// ============================================================================================
// Neighbour access (getPULeft / getPUAbove / getPUAboveLeft / getPUBelowLeft / getPUAboveRight)
// ============================================================================================
struct Nb { const Part *p; int idx; int valid; };
__device__ __forceinline__ const Part *ctu_parts(int addr) {
  HMC(addr >= 0 && addr < E.P.w_ctus * E.P.h_ctus, 1, addr, E.ctu_addr);
  if (HM_CHECKING && (addr < 0 || addr >= E.P.w_ctus * E.P.h_ctus)) addr = E.ctu_addr;
  return addr == E.ctu_addr ? E.S->ctu_p : E.P.ctus[addr].p;
}
// getCtuLeft / getCtuAbove / ... with CUIsFromSameSliceAndTile (TComDataCU.cpp:1024-1238)
__device__ __forceinline__ int ctu_in_slice(int a) { return a >= E.slice_start ? a : -1; }
__device__ __forceinline__ int ctu_left() { return E.ctu_x > 0 ? ctu_in_slice(E.ctu_addr - 1) : -1; }
__device__ __forceinline__ int ctu_above() { return E.ctu_y > 0 ? ctu_in_slice(E.ctu_addr - E.P.w_ctus) : -1; }
__device__ __forceinline__ int ctu_above_left() {
  return (E.ctu_x > 0 && E.ctu_y > 0) ? ctu_in_slice(E.ctu_addr - E.P.w_ctus - 1) : -1;
}
__device__ __forceinline__ int ctu_above_right() {
  return (E.ctu_y > 0 && E.ctu_x < E.P.w_ctus - 1) ? ctu_in_slice(E.ctu_addr - E.P.w_ctus + 1) : -1;
}
__device__ __forceinline__ Nb nb_none() { return Nb{nullptr, 0, 0}; }
__device__ __forceinline__ Nb nb_make(const Part *p, int idx) {
  HMC(idx >= 0 && idx < 256, 2, idx, 0);
  if (HM_CHECKING && (idx < 0 || idx >= 256)) idx = 0;
  return Nb{p, idx, 1};
}

__device__ Nb get_pu_left(const Cu *cu, int cur) {
  const int r = z2r(cur), rc = z2r(cu->zidx);
  if ((r & 15) != 0) {
    const int z = r2z(r - 1);
    if ((r & 15) == (rc & 15)) return nb_make(ctu_parts(E.ctu_addr), z);
    return nb_make(cu->p, z - cu->zidx);
  }
  const int a = ctu_left();
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(a), r2z(r + 15));
}
__device__ Nb get_pu_above(const Cu *cu, int cur, int planar_at_ctu_boundary) {
  const int r = z2r(cur), rc = z2r(cu->zidx);
  if ((r >> 4) != 0) {
    const int z = r2z(r - 16);
    if ((r >> 4) == (rc >> 4)) return nb_make(ctu_parts(E.ctu_addr), z);
    return nb_make(cu->p, z - cu->zidx);
  }
  if (planar_at_ctu_boundary) return nb_none();
  const int a = ctu_above();
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(a), r2z(r + 256 - 16));
}
__device__ Nb get_pu_above_left(const Cu *cu, int cur) {
  const int r = z2r(cur), rc = z2r(cu->zidx);
  if ((r & 15) != 0) {
    if ((r >> 4) != 0) {
      const int z = r2z(r - 17);
      if ((r & 15) == (rc & 15) || (r >> 4) == (rc >> 4)) return nb_make(ctu_parts(E.ctu_addr), z);
      return nb_make(cu->p, z - cu->zidx);
    }
    const int a = ctu_above();
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(a), r2z(r + 256 - 16 - 1));
  }
  if ((r >> 4) != 0) {
    const int a = ctu_left();
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(a), r2z(r - 1));
  }
  const int a = ctu_above_left();
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(a), r2z(255));
}
__device__ Nb get_pu_below_left(const Cu *cu, int cur, int off) {
  const int r = z2r(cur);
  const int rc_lb = z2r(cu->zidx) + ((cu->width >> 2) - 1) * 16;
  if (E.ctu_y * 64 + rpy(r) + 4 * off >= E.P.h) return nb_none();
  if ((r >> 4) < 16 - off) {
    if ((r & 15) != 0) {
      const int zz = r2z(r + off * 16 - 1);
      if (cur > zz) {
        if ((r & 15) == (rc_lb & 15) || (r >> 4) == (rc_lb >> 4)) return nb_make(ctu_parts(E.ctu_addr), zz);
        return nb_make(cu->p, zz - cu->zidx);
      }
      return nb_none();
    }
    const int a = ctu_left();
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(a), r2z(r + (1 + off) * 16 - 1));
  }
  return nb_none();
}
__device__ Nb get_pu_above_right(const Cu *cu, int cur, int off) {
  const int r = z2r(cur);
  const int rc_rt = z2r(cu->zidx) + (cu->width >> 2) - 1;
  if (E.ctu_x * 64 + rpx(r) + 4 * off >= E.P.w) return nb_none();
  if ((r & 15) < 16 - off) {
    if ((r >> 4) != 0) {
      const int zz = r2z(r - 16 + off);
      if (cur > zz) {
        if ((r & 15) == (rc_rt & 15) || (r >> 4) == (rc_rt >> 4)) return nb_make(ctu_parts(E.ctu_addr), zz);
        return nb_make(cu->p, zz - cu->zidx);
      }
      return nb_none();
    }
    const int a = ctu_above();
    if (a < 0) return nb_none();
    return nb_make(ctu_parts(a), r2z(r + 256 - 16 + off));
  }
  if ((r >> 4) != 0) return nb_none();
  const int a = ctu_above_right();
  if (a < 0) return nb_none();
  return nb_make(ctu_parts(a), r2z(256 - 16 + off - 1));
}
__device__ __forceinline__ int nb_inter(const Nb &n) { return n.valid && n.p[n.idx].pred == MODE_INTER; }

// ============================================================================================
// Partition geometry (getPartIndexAndSize, getPartPosition, derive*Idx, xDeriveCenterIdx)
// ============================================================================================
__device__ __forceinline__ int num_parts_of(int ps) { return ps == SIZE_2Nx2N ? 1 : ps == SIZE_NxN ? 4 : 2; }
__device__ __forceinline__ void part_index_size(const Cu *cu, int ps, int pu, int &addr, int &w, int &h) {
  const int W = cu->width, N = cu->nparts;
  switch (ps) {
    case SIZE_2NxN: w = W; h = W >> 1; addr = pu ? N >> 1 : 0; break;
    case SIZE_Nx2N: w = W >> 1; h = W; addr = pu ? N >> 2 : 0; break;
    case SIZE_NxN: w = W >> 1; h = W >> 1; addr = (N >> 2) * pu; break;
    case SIZE_2NxnU: w = W; h = pu ? (W >> 2) + (W >> 1) : W >> 2; addr = pu ? N >> 3 : 0; break;
    case SIZE_2NxnD: w = W; h = pu ? W >> 2 : (W >> 2) + (W >> 1); addr = pu ? (N >> 1) + (N >> 3) : 0; break;
    case SIZE_nLx2N: w = pu ? (W >> 2) + (W >> 1) : W >> 2; h = W; addr = pu ? N >> 4 : 0; break;
    case SIZE_nRx2N: w = pu ? W >> 2 : (W >> 2) + (W >> 1); h = W; addr = pu ? (N >> 2) + (N >> 4) : 0; break;
    default: w = W; h = W; addr = 0; break;
  }
}
__device__ __forceinline__ void part_position(const Cu *cu, int ps, int pu, int &xp, int &yp, int &w, int &h) {
  const int W = cu->width;
  int a;
  part_index_size(cu, ps, pu, a, w, h);
  xp = cu->x;
  yp = cu->y;
  switch (ps) {
    case SIZE_2NxN: case SIZE_2NxnU: case SIZE_2NxnD: yp = pu ? cu->y + W - h : cu->y; break;
    case SIZE_Nx2N: case SIZE_nLx2N: case SIZE_nRx2N: xp = pu ? cu->x + W - w : cu->x; break;
    case SIZE_NxN: xp = cu->x + (pu & 1) * w; yp = cu->y + (pu >> 1) * h; break;
    default: break;
  }
}
__device__ __forceinline__ void pu_corners(const Cu *cu, int ps, int pu, int &lt, int &rt, int &lb) {
  int a, w, h;
  part_index_size(cu, ps, pu, a, w, h);
  const int r = z2r(cu->zidx + a);
  lt = cu->zidx + a;
  rt = r2z(r + (w >> 2) - 1);
  lb = r2z(r + ((h >> 2) - 1) * 16);
}
__device__ __forceinline__ int pu_right_bottom(const Cu *cu, int ps, int pu) {
  int a, w, h;
  part_index_size(cu, ps, pu, a, w, h);
  return r2z(z2r(cu->zidx + a) + ((h >> 2) - 1) * 16 + (w >> 2) - 1);
}
__device__ __forceinline__ int pu_center(const Cu *cu, int ps, int pu) {
  int a, w, h;
  part_index_size(cu, ps, pu, a, w, h);
  return r2z(z2r(cu->zidx + a) + ((h >> 2) / 2) * 16 + (w >> 2) / 2);
}

// ============================================================================================
// Sub-part setters over a PU (TComDataCU::setSubPart family), lane-parallel
// ============================================================================================
template <class F>
__device__ __forceinline__ void pu_apply(Cu *cu, int ps, int pu, F f) {
  int a, w, h;
  part_index_size(cu, ps, pu, a, w, h);
  const int r0 = z2r(cu->zidx + a), nw = w >> 2, n = nw * (h >> 2);
  for (int i = lid(); i < n; i += 64) {
    const int y = i / nw, x = i - y * nw;
    f(cu->p[r2z(r0 + y * 16 + x) - cu->zidx]);
  }
  wsync();
}
__device__ void pu_set_mvfield(Cu *cu, int ps, int pu, int list, int mx, int my, int ref) {
  pu_apply(cu, ps, pu, [&](Part &p) { p.mv[list][0] = (int16_t)mx; p.mv[list][1] = (int16_t)my; p.ref[list] = (int8_t)ref; });
}
__device__ void pu_set_mv(Cu *cu, int ps, int pu, int list, int mx, int my) {
  pu_apply(cu, ps, pu, [&](Part &p) { p.mv[list][0] = (int16_t)mx; p.mv[list][1] = (int16_t)my; });
}
__device__ void pu_set_ref(Cu *cu, int ps, int pu, int list, int ref) {
  pu_apply(cu, ps, pu, [&](Part &p) { p.ref[list] = (int8_t)ref; });
}
__device__ void pu_set_mvd(Cu *cu, int ps, int pu, int list, int mx, int my) {
  pu_apply(cu, ps, pu, [&](Part &p) { p.mvd[list][0] = (int16_t)mx; p.mvd[list][1] = (int16_t)my; });
}
enum { PU_MERGE, PU_MERGE_IDX, PU_INTER_DIR, PU_MVP_IDX, PU_MVP_NUM };
__device__ void pu_set(Cu *cu, int ps, int pu, int which, int list, int v) {
  pu_apply(cu, ps, pu, [&](Part &p) {
    switch (which) {
      case PU_MERGE: p.merge = (int8_t)v; break;
      case PU_MERGE_IDX: p.merge_idx = (int8_t)v; break;
      case PU_INTER_DIR: p.inter_dir = (int8_t)v; break;
      case PU_MVP_IDX: p.mvp_idx[list] = (int8_t)v; break;
      default: p.mvp_num[list] = (int8_t)v; break;
    }
  });
}
enum { F_PART, F_PRED, F_SKIP, F_TRIDX };
__device__ void cu_set_all(Cu *cu, int field, int v) {
  const int n = cu->nparts;
  for (int i = lid(); i < n; i += 64) {
    Part &p = cu->p[i];
    if (field == F_PART) p.part = (int8_t)v;
    else if (field == F_PRED) p.pred = (int8_t)v;
    else if (field == F_SKIP) p.skip = (int8_t)v;
    else p.tr_idx = (int8_t)v;
  }
  wsync();
}
// a range of partitions [rel, rel + n): one byte field
__device__ void set_cbf_range(Cu *cu, int comp, int rel, int n, int v) {
  for (int i = lid(); i < n; i += 64) cu->p[rel + i].cbf[comp] = (uint8_t)v;
  wsync();
}
__device__ void or_cbf_range(Cu *cu, int comp, int rel, int n, int v) {
  for (int i = lid(); i < n; i += 64) cu->p[rel + i].cbf[comp] |= (uint8_t)v;
  wsync();
}
__device__ void set_ts_range(Cu *cu, int comp, int rel, int n, int v) {
  for (int i = lid(); i < n; i += 64) cu->p[rel + i].ts[comp] = (uint8_t)v;
  wsync();
}
__device__ void set_tridx(Cu *cu, int rel, int n, int v) {
  for (int i = lid(); i < n; i += 64) cu->p[rel + i].tr_idx = (int8_t)v;
  wsync();
}
__device__ void set_idir(Cu *cu, int ch, int rel, int n, int v) {
  for (int i = lid(); i < n; i += 64) cu->p[rel + i].idir[ch] = (uint8_t)v;
  wsync();
}

// initEstData (TComDataCU.cpp:552)
__device__ void cu_init_est(Cu *cu, int qp) {
  const int n = cu->nparts, depth = cu->depth, width = cu->width;
  for (int i = lid(); i < n; i += 64) {
    Part p;
    memset(&p, 0, sizeof(p));
    p.mvp_idx[0] = p.mvp_idx[1] = -1;
    p.mvp_num[0] = p.mvp_num[1] = -1;
    p.depth = (int8_t)depth;
    p.width = (uint8_t)width;
    p.part = SIZE_NONE;
    p.pred = MODE_NONE;
    p.qp = (int8_t)qp;
    p.idir[0] = 1;
    p.idir[1] = 0;
    p.ref[0] = p.ref[1] = -1;
    cu->p[i] = p;
  }
  const int ny = width * width;
  uint32_t *c0 = (uint32_t *)cu->coef;
  for (int i = lid(); i < (ny >> 1); i += 64) c0[i] = 0;
  uint32_t *c1 = (uint32_t *)(cu->coef + 4096), *c2 = (uint32_t *)(cu->coef + 5120);
  for (int i = lid(); i < (ny >> 3); i += 64) { c1[i] = 0; c2[i] = 0; }
  cu->bits = 0; cu->dist = 0; cu->cost = kMaxDouble; cu->dssim = 0;
  wsync();
}
// initSubCU (:623)
__device__ void cu_init_sub(Cu *cu, const Cu *parent, int idx, int depth, int qp) {
  const int pz = parent->zidx, pn = parent->nparts, px = parent->x, py = parent->y;
  wsync();
  cu->depth = depth;
  cu->width = 64 >> depth;
  cu->nparts = 256 >> (2 * depth);
  cu->zidx = pz + (pn >> 2) * idx;
  cu->x = px + (64 >> depth) * (idx & 1);
  cu->y = py + (64 >> depth) * (idx >> 1);
  cu_init_est(cu, qp);
}
// word copies (lane-parallel); byte counts are multiples of 4
__device__ __forceinline__ void copy_words(void *dst, const void *src, int bytes) {
  uint32_t *d = (uint32_t *)dst;
  const uint32_t *s = (const uint32_t *)src;
  for (int i = lid(); i < (bytes >> 2); i += 64) d[i] = s[i];
}
// copyPartFrom (:859)
__device__ void cu_copy_part_from(Cu *dst, const Cu *src, int idx, int depth) {
  const double sc = src->cost, ss = src->dssim;
  const uint32_t sd = src->dist, sb = src->bits;
  const int sn = src->nparts;
  wsync();
  dst->cost += sc;
  dst->dssim += ss;
  dst->dist += sd;
  dst->bits += sb;
  copy_words(&dst->p[sn * idx], src->p, (int)sizeof(Part) * sn);
  const int ny = (64 * 64) >> (depth << 1);
  copy_words(dst->coef + idx * ny, src->coef, 2 * ny);
  copy_words(dst->coef + 4096 + idx * (ny >> 2), src->coef + 4096, ny >> 1);
  copy_words(dst->coef + 5120 + idx * (ny >> 2), src->coef + 5120, ny >> 1);
  wsync();
}
// copyToPic (:945)
__device__ void cu_copy_to_pic(const Cu *cu) {
  State *S = E.S;
  const double c = cu->cost;
  const uint32_t d = cu->dist, b = cu->bits;
  const int z = cu->zidx, n = cu->nparts, depth = cu->depth;
  wsync();
  S->ctu_cost = c; S->ctu_dist = d; S->ctu_bits = b;
  copy_words(&S->ctu_p[z], cu->p, (int)sizeof(Part) * n);
  const int ny = (64 * 64) >> (depth << 1), off = z * 16;
  copy_words(S->ctu_coef + off, cu->coef, 2 * ny);
  copy_words(S->ctu_coef + 4096 + (off >> 2), cu->coef + 4096, ny >> 1);
  copy_words(S->ctu_coef + 5120 + (off >> 2), cu->coef + 5120, ny >> 1);
  wsync();
}
__device__ __forceinline__ int cu_qt_root_cbf(const Cu *cu, int i) {
  return (cu->p[i].cbf[0] & 1) || (cu->p[i].cbf[1] & 1) || (cu->p[i].cbf[2] & 1);
}
__device__ __forceinline__ int cbf_at(const Part *p, int comp, int depth) { return (p->cbf[comp] >> depth) & 1; }
#ifdef HM_CHECKS
// the header of a CU object is consistent (a debugging aid: finds writes that clobber it)
__device__ void cu_sane(const Cu *cu, int code) {
  const int d = cu->depth;
  const bool ok = d >= 0 && d < 4 && cu->width == (64 >> d) && cu->nparts == (256 >> (2 * d)) && cu->zidx >= 0 && cu->zidx < 256;
  HMC(ok, code, d, (int)((const char *)cu - (const char *)E.S->cu));
}
#define HMCU(cu, code) cu_sane((cu), (code))
#else
#define HMCU(cu, code) ((void)0)
#endif

// ============================================================================================
// Syntax elements (TEncSbac.cpp:427-1104) on a bin sink: the RD counter of the decision
// (CountSink: TEncBinCABACCounter on E.cod[E.cur], only the number of bypass bins matters) or the
// slice writer (hvx_hmwrite.hpp: TEncBinCABAC, the bypass bins' values written msb first)
// ============================================================================================
struct CountSink {
  static constexpr bool kValues = false;  // the bypass bins' values are not needed
  __device__ __forceinline__ void bin(int ctx, int v) const { cbin(ctx, v); }
  __device__ __forceinline__ void eps(uint32_t, int n) const { cep(n); }
  __device__ __forceinline__ void trm(int v) const { ctrm(v); }
};
template <class K = CountSink>
__device__ void code_split_flag(const Cu *cu, int rel, int depth, K k = K()) {
  if (depth == 3) return;
  const Nb l = get_pu_left(cu, cu->zidx + rel), a = get_pu_above(cu, cu->zidx + rel, 0);
  const int ctx = (l.valid && l.p[l.idx].depth > depth) + (a.valid && a.p[a.idx].depth > depth);
  k.bin(X_SPLIT + ctx, cu->p[rel].depth > depth);
}
template <class K = CountSink>
__device__ void code_skip_flag(const Cu *cu, int rel, K k = K()) {
  if (E.P.slice_type == I_SLICE) return;
  const Nb l = get_pu_left(cu, cu->zidx + rel), a = get_pu_above(cu, cu->zidx + rel, 0);
  const int ctx = (l.valid && l.p[l.idx].skip) + (a.valid && a.p[a.idx].skip);
  k.bin(X_SKIP + ctx, cu->p[rel].skip ? 1 : 0);
}
template <class K = CountSink>
__device__ void code_merge_index(const Cu *cu, int rel, K k = K()) {
  const int idx = cu->p[rel].merge_idx, n = E.P.max_merge;
  if (n > 1)
    for (int i = 0; i < n - 1; i++) {
      const int sym = i == idx ? 0 : 1;
      if (i == 0) k.bin(X_MERGE_IDX, sym);
      else k.eps((uint32_t)sym, 1);
      if (!sym) break;
    }
}
template <class K = CountSink>
__device__ void code_pred_mode(const Cu *cu, int rel, K k = K()) {
  if (E.P.slice_type == I_SLICE) return;
  k.bin(X_PRED, cu->p[rel].pred == MODE_INTRA);
}
template <class K = CountSink>
__device__ void code_part_size(const Cu *cu, int rel, int depth, K k = K()) {
  const int ps = cu->p[rel].part;
  if (cu->p[rel].pred == MODE_INTRA) {
    if (depth == 3) k.bin(X_PART + 0, ps == SIZE_2Nx2N);
    return;
  }
  const int amp = E.P.amp && depth < 3;
  switch (ps) {
    case SIZE_2Nx2N: k.bin(X_PART + 0, 1); break;
    case SIZE_2NxN: case SIZE_2NxnU: case SIZE_2NxnD:
      k.bin(X_PART + 0, 0);
      k.bin(X_PART + 1, 1);
      if (amp) {
        if (ps == SIZE_2NxN) k.bin(X_PART + 3, 1);
        else { k.bin(X_PART + 3, 0); k.eps(ps == SIZE_2NxnU ? 0u : 1u, 1); }
      }
      break;
    case SIZE_Nx2N: case SIZE_nLx2N: case SIZE_nRx2N:
      k.bin(X_PART + 0, 0);
      k.bin(X_PART + 1, 0);
      if (depth == 3 && cu->p[rel].width != 8) k.bin(X_PART + 2, 1);
      if (amp) {
        if (ps == SIZE_Nx2N) k.bin(X_PART + 3, 1);
        else { k.bin(X_PART + 3, 0); k.eps(ps == SIZE_nLx2N ? 0u : 1u, 1); }
      }
      break;
    case SIZE_NxN:
      if (depth == 3 && cu->p[rel].width != 8) { k.bin(X_PART + 0, 0); k.bin(X_PART + 1, 0); k.bin(X_PART + 2, 0); }
      break;
    default: break;
  }
}
// getIntraDirPredictor (TComDataCU.cpp:1401): the three most probable luma modes of a PU
__device__ void intra_mpm_list(const Cu *cu, int rel, int p[3]) {
  const Nb l = get_pu_left(cu, cu->zidx + rel), a = get_pu_above(cu, cu->zidx + rel, 1);
  const int ld = (l.valid && l.p[l.idx].pred == MODE_INTRA) ? l.p[l.idx].idir[0] : 1;
  const int ad = (a.valid && a.p[a.idx].pred == MODE_INTRA) ? a.p[a.idx].idir[0] : 1;
  if (ld == ad) {
    if (ld > 1) { p[0] = ld; p[1] = ((ld + 29) % 32) + 2; p[2] = ((ld - 1) % 32) + 2; }
    else { p[0] = 0; p[1] = 1; p[2] = 26; }
  } else {
    p[0] = ld; p[1] = ad;
    p[2] = (ld && ad) ? 0 : ((ld + ad) < 2 ? 26 : 1);
  }
}
// codeIntraDirLumaAng (:643): the MPM flags of the PUs, then per PU the MPM index (truncated
// unary, bypass) or the 5-bit remaining mode (the MPMs sorted and stepped over)
template <class K = CountSink>
__device__ void code_intra_dir_luma(const Cu *cu, int rel, int multiple, K k = K()) {
  const int npu = (multiple && cu->p[rel].part == SIZE_NxN) ? 4 : 1;
  const int off = (256 >> (2 * cu->p[rel].depth)) >> 2;
  int pidx[4] = {-1, -1, -1, -1}, rem[4] = {0, 0, 0, 0};
  for (int j = 0; j < npu; j++) {
    int p[3];
    intra_mpm_list(cu, rel + off * j, p);
    int dir = cu->p[rel + off * j].idir[0], pi = -1;
    for (int i = 0; i < 3; i++)
      if (dir == p[i]) pi = i;
    if (K::kValues && pi < 0) {
      if (p[0] > p[1]) { const int t = p[0]; p[0] = p[1]; p[1] = t; }
      if (p[0] > p[2]) { const int t = p[0]; p[0] = p[2]; p[2] = t; }
      if (p[1] > p[2]) { const int t = p[1]; p[1] = p[2]; p[2] = t; }
      for (int i = 2; i >= 0; i--) dir = dir > p[i] ? dir - 1 : dir;
      rem[j] = dir;
    }
    pidx[j] = pi;
    k.bin(X_INTRA, pi != -1);
  }
  for (int j = 0; j < npu; j++) {
    if (pidx[j] != -1) {
      if (pidx[j]) k.eps(2u | (uint32_t)(pidx[j] - 1), 2);
      else k.eps(0u, 1);
    } else k.eps((uint32_t)rem[j], 5);
  }
}
// codeIntraDirChroma (:700): DM, or the index among getAllowedChromaDir's first four
template <class K = CountSink>
__device__ void code_intra_dir_chroma(const Cu *cu, int rel, K k = K()) {
  const int dc = cu->p[rel].idir[1];
  if (dc == DM_CHROMA_IDX) { k.bin(X_CHROMA, 0); return; }
  k.bin(X_CHROMA, 1);
  int sym = 0;
  if constexpr (K::kValues) {
    const int lm = cu->p[rel].idir[0];
    int allowed[4] = {0, 26, 10, 1};
    for (int i = 0; i < 4; i++)
      if (allowed[i] == lm) { allowed[i] = 34; break; }
    for (int i = 0; i < 4; i++)
      if (dc == allowed[i]) { sym = i; break; }
  }
  k.eps((uint32_t)sym, 2);
}
template <class K = CountSink>
__device__ void code_ref_idx(const Cu *cu, int rel, int list, K k = K()) {
  int r = cu->p[rel].ref[list];
  k.bin(X_REF + 0, r == 0 ? 0 : 1);
  if (r > 0) {
    const int n = E.P.nref[list] - 2;
    r--;
    for (int i = 0; i < n; i++) {
      const int sym = i == r ? 0 : 1;
      if (i == 0) k.bin(X_REF + 1, sym);
      else k.eps((uint32_t)sym, 1);
      if (!sym) break;
    }
  }
}
// xWriteEpExGolomb (TEncSbac.cpp:307): the k-th order Exp-Golomb code of sym as one bypass string
template <class K>
__device__ __forceinline__ void ep_exgolomb(uint32_t sym, int count, K k) {
  uint32_t bins = 0;
  int n = 0;
  while (sym >= (1u << count)) { bins = 2 * bins + 1; n++; sym -= 1u << count; count++; }
  bins = 2 * bins;
  n++;
  bins = (bins << count) | sym;
  n += count;
  k.eps(bins, n);
}
template <class K = CountSink>
__device__ void code_mvd(const Cu *cu, int rel, int list, K k = K()) {
  if (E.P.mvd_l1_zero && list == 1 && cu->p[rel].inter_dir == 3) return;  // TEncSbac.cpp:781
  const int h = cu->p[rel].mvd[list][0], v = cu->p[rel].mvd[list][1];
  k.bin(X_MVD + 0, h != 0);
  k.bin(X_MVD + 0, v != 0);
  const int ah = abs(h), av = abs(v);
  if (h) k.bin(X_MVD + 1, ah > 1);
  if (v) k.bin(X_MVD + 1, av > 1);
  if (h) { if (ah > 1) ep_exgolomb((uint32_t)(ah - 2), 1, k); k.eps(h < 0 ? 1u : 0u, 1); }
  if (v) { if (av > 1) ep_exgolomb((uint32_t)(av - 2), 1, k); k.eps(v < 0 ? 1u : 0u, 1); }
}
template <class K = CountSink>
__device__ void code_inter_dir(const Cu *cu, int rel, K k = K()) {
  const int d = cu->p[rel].inter_dir - 1, ctx = cu->p[rel].depth;
  if (cu->p[rel].part == SIZE_2Nx2N || cu->p[rel].width != 8) k.bin(X_INTER_DIR + ctx, d == 2);
  if (d < 2) k.bin(X_INTER_DIR + 4, d);
}
template <class K = CountSink>
__device__ void encode_pu_wise(const Cu *cu, int rel, K k = K()) {
  const int ps = cu->p[rel].part, npu = num_parts_of(ps);
  const int off16 = ps == 0 ? 0 : ps == 1 ? 8 : ps == 2 ? 4 : ps == 3 ? 4 : ps == 4 ? 2 : ps == 5 ? 10 : ps == 6 ? 1 : 5;
  const int puoff = (off16 << ((4 - cu->p[rel].depth) << 1)) >> 4;
  for (int pu = 0, sub = rel; pu < npu; pu++, sub += puoff) {
    k.bin(X_MERGE_FLAG, cu->p[sub].merge ? 1 : 0);
    if (cu->p[sub].merge) code_merge_index(cu, sub, k);
    else {
      if (E.P.slice_type == B_SLICE) code_inter_dir(cu, sub, k);
      for (int l = 0; l < 2; l++)
        if (E.P.nref[l] > 0) {
          const int dir = cu->p[sub].inter_dir;
          if (E.P.nref[l] != 1 && (dir & (1 << l))) code_ref_idx(cu, sub, l, k);
          if (dir & (1 << l)) code_mvd(cu, sub, l, k);
          if (dir & (1 << l)) k.bin(X_MVP, cu->p[sub].mvp_idx[l] ? 1 : 0);
        }
    }
  }
}
template <class K = CountSink>
__device__ void encode_pred_info(const Cu *cu, int rel, K k = K()) {
  if (cu->p[rel].pred == MODE_INTRA) {
    code_intra_dir_luma(cu, rel, 1, k);
    code_intra_dir_chroma(cu, rel, k);
  } else encode_pu_wise(cu, rel, k);
}

// ============================================================================================
// Transform-unit recursion: TComTU / TComTURecurse, 4:2:0 (rectangles relative to the CU)
// ============================================================================================
__device__ __forceinline__ void tu_root(Tu &t, const Cu *cu, int init_tr_depth) {
  const int depth = cu->depth, zidx = cu->zidx, width = cu->width;
  t.cu_depth = depth;
  t.cu_zidx = zidx;
  t.split = 0;
  t.section = 0;
  t.last_of_level = 1;
  t.rel = 0;
  t.step = 256 >> (2 * depth);
  int l = 0;
  while ((4 << l) < (64 >> (depth + init_tr_depth))) l++;
  t.log2 = l + 2;
  for (int c = 0; c < 3; c++) {
    t.trd[c] = init_tr_depth;
    t.x0[c] = t.y0[c] = 0;
    t.w[c] = t.h[c] = t.ow[c] = c ? width >> 1 : width;
    t.all[c] = 1;
    t.off[c] = 0;
  }
}
__device__ __forceinline__ void tu_child(Tu &t, const Tu &p, int last_of_level) {
  t = p;
  t.split = 2;
  t.section = 0;
  t.last_of_level = last_of_level;
  t.rel = p.all[0] ? p.rel : (p.rel & ~3);
  t.step = (p.step >> 2) > 1 ? p.step >> 2 : 1;
  t.log2 = p.log2 - 1;
  for (int c = 0; c < 3; c++) {
    t.trd[c] = p.trd[c] + 1;
    t.w[c] = p.w[c] >> 1;
    t.h[c] = p.h[c] >> 1;
    t.x0[c] = p.x0[c];
    t.y0[c] = p.y0[c];
    t.off[c] = p.off[c];
    if ((t.w[c] < 4 || t.h[c] < 4) && t.w[c] != 0) {
      t.w[c] = p.w[c];
      t.h[c] = p.h[c];
      t.all[c] = 0;
      t.trd[c]--;
    } else t.all[c] = 1;
    t.ow[c] = t.w[c];
    if (!t.all[c] && last_of_level) t.w[c] = 0;
  }
}
__device__ __forceinline__ int tu_next(Tu &t, const Tu &p) {
  for (int c = 0; c < 3; c++) {
    t.off[c] += t.w[c] * t.h[c];
    if (t.last_of_level) t.w[c] = t.ow[c];
    t.x0[c] += t.w[c];
    if (t.x0[c] >= p.x0[c] + p.w[c]) { t.x0[c] = p.x0[c]; t.y0[c] += t.h[c]; }
    if (!t.all[c] && (!t.last_of_level || t.section != 2)) t.w[c] = 0;
  }
  t.rel += t.step;
  t.section++;
  return t.section < 4;
}
__device__ __forceinline__ int tu_abs_rel(const Tu &t) { return t.rel; }
__device__ __forceinline__ int tu_abs_rel_c(const Tu &t, int c) { return t.all[c] ? t.rel : (t.rel & ~3); }
__device__ __forceinline__ int tu_nparts(const Tu &t, int c) { return t.all[c] ? t.step : t.step * 4; }
__device__ __forceinline__ int tu_proc(const Tu &t, int c) { return t.w[c] != 0; }
__device__ __forceinline__ int tu_depth_rel(const Tu &t) { return t.trd[0]; }
__device__ __forceinline__ int tu_depth_total(const Tu &t) { return t.cu_depth + t.trd[0]; }
__device__ __forceinline__ int qt_layer(int log2) { return 5 - log2; }

// getQuadtreeTULog2MinSizeInCU (TComDataCU.cpp:1518)
__device__ int qt_min_log2(const Cu *cu, int rel) {
  const int l2 = ilog2(cu->width);
  const int isplit = (cu->p[rel].pred == MODE_INTRA && cu->p[rel].part == SIZE_NxN) ? 1 : 0;
  if (l2 < 2 + 3 - 1 + isplit) return 2;
  const int m = l2 - (3 - 1 + isplit);
  return m > 5 ? 5 : m;
}
template <class K = CountSink>
__device__ void code_qt_cbf(const Cu *cu, const Tu &t, int comp, int lowest, K k = K()) {
  const int ch = comp ? 1 : 0;
  const int depth = tu_depth_rel(t);
  const int ctx = ch ? depth : (depth == 0 ? 1 : 0);
  const int can_split = t.w[comp] >= 8 && t.h[comp] >= 8;
  const int lowest_depth = depth + ((!lowest && !can_split) ? 1 : 0);
  k.bin(X_QT_CBF + ch * 5 + ctx, cbf_at(&cu->p[tu_abs_rel_c(t, comp)], comp, lowest_depth));
}
__device__ void code_qt_cbf_zero(const Tu &t, int ch) {
  const int depth = tu_depth_rel(t);
  cbin(X_QT_CBF + ch * 5 + (ch ? depth : (depth == 0 ? 1 : 0)), 0);
}
__device__ __forceinline__ void code_subdiv(int v, int ctx) { cbin(X_SUBDIV + ctx, v); }

// getCoefScanIdx (TComDataCU.cpp:3177), 4:2:0
__device__ int coef_scan_idx(const Cu *cu, int rel, int w, int comp) {
  if (cu->p[rel].pred != MODE_INTRA) return 0;
  const int maxw = comp ? 4 : 8;
  if (w > maxw) return 0;
  int dir = cu->p[rel].idir[comp ? 1 : 0];
  if (dir == DM_CHROMA_IDX) dir = cu->p[comp ? (rel & ~3) : rel].idir[0];
  if (abs(dir - 26) <= 4) return 1;
  if (abs(dir - 10) <= 4) return 2;
  return 0;
}
// the descriptor of the TU a transform / count / inverse works on (wave-uniform, one at a time):
// E.td in LDS -- a per-lane copy lived in scratch (7 KB of call-frame traffic per TU call)
__device__ void tu_desc(const Cu *cu, const Tu &t, int comp) {
  hvx_tu_desc &d = E.td;
  const int rel = tu_abs_rel_c(t, comp);
  const int scan = coef_scan_idx(cu, rel, t.w[comp], comp);
  const int intra = cu->p[rel].pred == MODE_INTRA;
  const int ts = cu->p[rel].ts[comp], tr = cu->p[rel].tr_idx;
  const int qp = comp ? E.P.chroma_qp[comp - 1] : E.slice_qp;
  const double lam = E.P.tq_lambda[comp];
  d.comp = comp;
  d.width = t.w[comp];
  d.height = t.h[comp];
  d.log2_size = ilog2(t.h[comp]);
  d.scan_type = scan;
  d.use_dst = comp == 0 && intra && t.w[0] == 4;
  d.transform_skip = ts;
  d.is_intra = intra;
  d.tr_idx = tr;
  d.ctx_qt_cbf = comp ? tu_depth_rel(t) : (tu_depth_rel(t) == 0 ? 1 : 0);
  d.slice_type = E.P.slice_type;
  d.qp_per = qp / 6;
  d.qp_rem = qp % 6;
  d.sign_hiding = 1;
  d.use_rdoq = d.use_rdoq_ts = 1;
  d.selective_rdoq = d.adaptive_qp_select = d.transquant_bypass = 0;
  d.golomb_rice_stat = d.persistent_rice = d.extended_precision = d.ts_context = 0;
  d.max_log2_tr_range = 15;
  d.bit_depth = 8;
  d.pps_tskip = 1;
  d.lambda = lam;
}
// the scan geometry of a TU (cab::ScanTables' values): the CG scan staged in LDS for every size;
// raster positions and packed significance contexts staged in LDS up to 16x16, while a 32x32 TU
// (big) reads its rasters from the constant scan table and derives the contexts per lane
struct StagedScan {
  const uint8_t *cgs;
  const int16_t *ras;
  const int32_t *sig;
  const uint16_t *scan_g;
  int first_sig, single;
  bool big;
  __device__ __forceinline__ int cg(int sub) const { return uni(cgs[sub]); }
  __device__ __forceinline__ int raster(int sp) const { return big ? (int)scan_g[sp] : uni(ras[sp]); }
  __device__ __forceinline__ int sigc(int pattern, int sp) const { return (uni(sig[sp]) >> (6 * pattern)) & 63; }
};

// cab::coeff_bits_env (codeCoeffNxN under the counter, TEncSbac.cpp:1181-1540) restated for the
// wave-uniform engine over a TU staged in scan order (every size): the same bins in the same order
// on the same contexts, but the significant-CG map is one ballot per 64 positions, and a
// coefficient group's levels and significance contexts are fetched lane-parallel once (one LDS
// round) and read back with v_readlane; the greater-1 / escape passes walk the set bits of the
// group's mask instead of all 16 positions.  One instance serves all sizes (a second walk in
// code_coeff_nxn costs registers across the whole function).  Returns num_sig.
template <class C>
__device__ int coeff_count_staged(const hvx_tu_desc &d, const StagedScan &env, const int16_t *ls, C &L) {
  const int n = d.width, lw = cab::log2_tu(n), wg = n >> 2, ncg = wg * wg, nn = n * n;
  const int ch = d.comp ? 1 : 0, l = lid();
  HM_WT0(wt_);
  // significant-CG map, count and last position: one ballot per 64 scan positions (4 groups)
  uint64_t cgm = 0;
  int num_sig = 0, scan_last = -1;
  const int nw = nn < 64 ? 1 : nn >> 6;
  for (int w = 0; w < nw; w++) {
    const uint64_t b = __ballot(w * 64 + l < nn && ls[w * 64 + l] != 0);
    if (b) {
      num_sig += __popcll(b);
      scan_last = w * 64 + 63 - __clzll(b);
#pragma unroll
      for (int q = 0; q < 4; q++)
        if ((b >> (16 * q)) & 0xffffu) cgm |= 1ull << env.cg(w * 4 + q);
    }
  }
  (void)ncg;
  if (num_sig == 0) return 0;
  const bool be_valid = d.transquant_bypass ? false : (d.sign_hiding != 0);
  if (d.pps_tskip && !d.transquant_bypass && n <= 4) L.bin(cab::kTskip + ch, d.transform_skip ? 1 : 0);
  {  // codeLastSignificantXY (:1115)
    const int r = env.raster(scan_last);
    int py = r >> lw, px = r - (py << lw);
    if (d.scan_type == 2) { const int t = px; px = py; py = t; }
    const int gx = kGroupIdx[px], gy = kGroupIdx[py], gmax = kGroupIdx[n - 1];
    const int cw = lw - 2;
    const int off = ch ? 0 : cw * 3 + ((cw + 1) >> 2), sh = ch ? cw : (cw + 3) >> 2;
    const int bx = cab::kLastX + ch * 15 + off, by = cab::kLastY + ch * 15 + off;
    int k;
    for (k = 0; k < gx; k++) L.bin(bx + (k >> sh), 1);
    if (gx < gmax) L.bin(bx + (k >> sh), 0);
    for (k = 0; k < gy; k++) L.bin(by + (k >> sh), 1);
    if (gy < gmax) L.bin(by + (k >> sh), 0);
    if (gx > 3) L.ep((gx - 2) >> 1);
    if (gy > 3) L.ep((gy - 2) >> 1);
  }
  HM_WTADD(0, wt_);
  const int base_cg = cab::kSigCG + ch * 2, base_sig = cab::kSig + (ch ? 28 : 0);
  const int last_set = scan_last >> 4, last_pin = scan_last & 15;
  int c1 = 1;
  for (int sub = last_set; sub >= 0; sub--) {
    const int sub_pos = sub << 4;
    const int cg = env.cg(sub), cgy = cg / wg, cgx = cg - cgy * wg;
    // the group's levels and significance-context words (32x32: raster positions), one position
    // per lane
    const int lv_l = l < 16 ? (int)ls[sub_pos + l] : 0;
    const int av_l = lv_l < 0 ? -lv_l : lv_l;
    const int sc_l = l < 16 ? (env.big ? (int)env.scan_g[sub_pos + l] : env.sig[sub_pos + l]) : 0;
    if (sub == last_set || sub == 0) cgm |= 1ull << cg;
    else {
      const int rr = cgx < wg - 1 ? (int)((cgm >> (cg + 1)) & 1) : 0;
      const int bb = cgy < wg - 1 ? (int)((cgm >> (cg + wg)) & 1) : 0;
      L.bin(base_cg + ((rr + bb) != 0), (int)((cgm >> cg) & 1));
    }
    const bool is_last_set = sub == last_set;
    const uint32_t m16 = (uint32_t)__ballot(lv_l != 0);
    if ((cgm >> cg) & 1) {
      int pattern = 0;
      if (wg > 1) {
        const int rr = cgx < wg - 1 ? (int)((cgm >> (cg + 1)) & 1) : 0;
        const int bb = cgy < wg - 1 ? (int)((cgm >> (cg + wg)) & 1) : 0;
        pattern = rr + (bb << 1);
      }
      const int sc = env.big ? cab::sig_ctx(pattern, env.first_sig, env.single, sc_l, lw, ch) : (sc_l >> (6 * pattern)) & 63;
      int nnz = is_last_set ? 1 : 0;
      // the group's significance contexts fetched into lanes once (one LDS round) and written back
      // once: a flag's bin reads its state with v_readlane and forwards the new state to every lane
      // on the same context, leaving one LDS round (the tables) on the chain per bin
      const int row_l = base_sig + (l < 16 ? sc : 0) + cab::kCtxLo;
      int q_l = L.st[row_l];
      for (int pin = is_last_set ? last_pin - 1 : 15; pin >= 0; pin--) {
        const int sig = (int)((m16 >> pin) & 1u);
        if (pin > 0 || sub == 0 || nnz) {
          const int row = __builtin_amdgcn_readlane(row_l, pin), q = __builtin_amdgcn_readlane(q_l, pin);
          const uint32_t pv = E.pk[q * 2 + sig];
          L.frac += pv & 0xffffffu;
          const int ns = (int)(pv >> 24);
          q_l = row_l == row ? ns : q_l;
        }
        nnz += sig;
      }
      if (l < 16) L.st[row_l] = (uint8_t)q_l;
    }
    const int nnz = __popc(m16);
    HM_WTADD(1, wt_);
    if (nnz == 0) continue;
    // greater-1 / greater-2 over the group's non-zero levels in reverse scan order (first 8)
    const int last_nz = 31 - __clz(m16), first_nz = __builtin_ctz(m16);
    const bool hidden = (last_nz - first_nz) >= 4;  // SBH_THRESHOLD
    const int set = (ch ? 4 : 0) + ((!ch && sub > 0) ? 2 : 0) + (c1 == 0 ? 1 : 0);
    c1 = 1;
    const int base_one = cab::kOne + 4 * set;
    bool escape = nnz > 8;
    int first_c2_abs = 0;
    bool have_c2 = false;
    uint32_t rest = m16;
    // the four greater-1 contexts of the set in lanes 0..3, the same way
    const int row1_l = base_one + (l & 3) + cab::kCtxLo;
    int q1_l = L.st[row1_l];
    for (int idx = 0; rest && idx < 8; idx++) {
      const int pin = 31 - __clz(rest);
      rest &= ~(1u << pin);
      const int av = __builtin_amdgcn_readlane(av_l, pin);
      const int gt1 = av > 1;
      {
        const int q = __builtin_amdgcn_readlane(q1_l, c1);
        const uint32_t pv = E.pk[q * 2 + gt1];
        L.frac += pv & 0xffffffu;
        const int ns = (int)(pv >> 24);
        q1_l = (l & 3) == c1 ? ns : q1_l;
      }
      if (gt1) {
        c1 = 0;
        if (!have_c2) { have_c2 = true; first_c2_abs = av; }
        else escape = true;
      } else if (c1 < 3 && c1 > 0) {
        c1++;
      }
    }
    if (l < 4) L.st[row1_l] = (uint8_t)q1_l;
    if (c1 == 0 && have_c2) {
      const int gt2 = first_c2_abs > 2;
      L.bin(cab::kAbs + set, gt2);
      if (gt2) escape = true;
    }
    HM_WTADD(2, wt_);
    L.ep((be_valid && hidden) ? nnz - 1 : nnz);  // signs (the first one hidden)
    if (escape) {
      // the escape codes' bin counts lane-parallel (bypass bins: only their total counts): a level's
      // base (idx < 8 ? 2 + first2 : 1) from the set bits before it; the Rice parameter (from 0, no
      // persistent adaptation in the engine's tool set) moves only at a level > 3 << rice, which is
      // always >= base, so it is scanned over the levels > 3 alone
      const int pin_l = l & 15;
      const uint32_t before = m16 & ~((2u << pin_l) - 1u);
      const uint32_t ge2 = (uint32_t)__ballot(l < 16 && av_l >= 2);
      const int base_l = __popc(before) < 8 ? 2 + ((ge2 & before) ? 0 : 1) : 1;
      int rice_l = 0;
      uint32_t big = (uint32_t)__ballot(l < 16 && av_l > 3);
      if (big) {
        int r = 0;
        while (big) {
          const int p = 31 - __clz(big);
          big &= ~(1u << p);
          if (__builtin_amdgcn_readlane(av_l, p) > (3 << r)) r = r + 1 < 4 ? r + 1 : 4;
          if (pin_l < p) rice_l = r;
        }
      }
      const uint32_t nb = l < 16 && av_l >= base_l
                              ? (uint32_t)cab::remain_bins((uint32_t)(av_l - base_l), rice_l, d.extended_precision != 0,
                                                           d.max_log2_tr_range)
                              : 0u;
      L.ep((int)wave_sum_u32(nb));
    }
    HM_WTADD(3, wt_);
  }
  return num_sig;
}

// codeCoeffNxN on the current coder, levels TU-packed int16.  The whole wave first stages the TU
// in LDS in scan order -- levels, raster positions, the significance context of every position
// under the four neighbour-CG patterns, the CG scan -- with one round of table and level loads;
// the serial syntax walk then reads LDS only (no global-memory latency on its chain).
// the byte mask of dword k (rows 40 + 4k .. 43 + 4k) over the context rows codeCoeffNxN of channel
// ch touches (TEncSbac.cpp:62-92: significant-CG, significance, last X / Y, greater-1, greater-2,
// transform skip)
__device__ __forceinline__ uint32_t memo_mask(int ch, int k) {
  uint32_t m = 0;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const int r = 40 + 4 * k + b;
    const bool in = ch ? ((r >= 44 && r <= 45) || (r >= 74 && r <= 89) || (r >= 105 && r <= 119) || (r >= 135 && r <= 149) ||
                          (r >= 166 && r <= 173) || (r >= 178 && r <= 179) || r == 184)
                       : ((r >= 42 && r <= 43) || (r >= 46 && r <= 72) || (r >= 90 && r <= 104) || (r >= 120 && r <= 134) ||
                          (r >= 150 && r <= 165) || (r >= 174 && r <= 177) || r == 183);
    m |= in ? 0xffu << (8 * b) : 0u;
  }
  return m;
}

// the memo index's content hash: murmur3-mixed lane words (masked context-state dwords, packed
// levels) summed over the wave
__device__ __forceinline__ uint32_t memo_mix(uint32_t x) {
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t memo_hash(uint32_t st_masked, uint32_t cf) {
  const uint32_t l = (uint32_t)lid();
  return wave_sum_u32(memo_mix(st_masked ^ (l * 0x9e3779b9u)) + memo_mix(cf ^ (l * 0x7f4a7c15u + 0x2545f491u)));
}
// desc_ready: E.td already describes this TU and component (the caller's transformNxN just made it)
__device__ void code_coeff_nxn(const Cu *cu, const Tu &t, int comp, const int16_t *coef, bool desc_ready = false) {
  HM_PROF(PR_COEF);
  HM_T0(t_desc);
  if (!desc_ready) tu_desc(cu, t, comp);
  const hvx_tu_desc &d = E.td;
  HM_TADD(PR_COEF_DESC, t_desc);
  // the memo (4x4 / 8x8 TUs)
  const int ch = comp ? 1 : 0, l = lid();
  const bool memo_on = d.width <= 8;
  uint32_t cur_st = 0, cur_cf = 0, mask = 0, key = 0, hash = 0;
  State *S = E.S;
  if (memo_on) {
    key = 0x8000u | (uint32_t)d.width | ((uint32_t)ch << 8) | ((uint32_t)d.scan_type << 10) | ((uint32_t)d.transform_skip << 12);
    const int ndw = d.width * d.width / 2;
    uint32_t *st32 = reinterpret_cast<uint32_t *>(E.cod[E.cur].st);
    if (l < kMemoDw) { cur_st = st32[kMemoDw0 + l]; mask = memo_mask(ch, l); }
    if (l < ndw) cur_cf = reinterpret_cast<const uint32_t *>(coef)[l];
    // the index in LDS: keys and a hash of the levels and masked context states; only an entry whose
    // hash matches is read from HBM, and compared in full there (a hash is never trusted alone)
    hash = memo_hash(cur_st & mask, cur_cf);
    uint64_t cand = __ballot(l < kMemoK && E.memo_key[l < kMemoK ? l : 0] == key && E.memo_hash[l < kMemoK ? l : 0] == hash);
    while (cand) {
      const int e = __builtin_ctzll(cand);
      cand &= cand - 1;
      const CoefMemo &m = S->memo[e];
      const uint32_t after = l < kMemoDw ? m.after[l] : 0u;  // read with the comparands (one round)
      const uint64_t f = m.frac;
      const bool diff = (l < kMemoDw && ((m.before[l] ^ cur_st) & mask)) || (l < ndw && m.coef[l] != cur_cf);
      if (__ballot(diff) == 0) {  // a repeat: replay its result
        wsync();
        if (l < kMemoDw) st32[kMemoDw0 + l] = (cur_st & ~mask) | (after & mask);
        if (l == 0) E.cod[E.cur].frac += f;
        wsync();
        return;
      }
    }
  }
  int bslot = -1;
  if (d.width >= 16) {  // the 16x16 / 32x32 memo: same index scheme, levels compared from registers
    key = 0x8000u | (uint32_t)d.width | ((uint32_t)ch << 8) | ((uint32_t)d.scan_type << 10) | ((uint32_t)d.transform_skip << 12);
    const int nper = d.width == 16 ? 2 : 8;
    uint32_t *st32 = reinterpret_cast<uint32_t *>(E.cod[E.cur].st);
    if (l < kMemoDw) { cur_st = st32[kMemoDw0 + l]; mask = memo_mask(ch, l); }
    const uint32_t *c32 = reinterpret_cast<const uint32_t *>(coef);
    uint32_t cf[8];
    uint32_t hs = memo_mix((cur_st & mask) ^ ((uint32_t)l * 0x9e3779b9u));
#pragma unroll
    for (int k = 0; k < 8; k++) {
      cf[k] = 0;
      if (k < nper) {
        cf[k] = c32[k * 64 + l];
        hs += memo_mix(cf[k] ^ ((uint32_t)(k * 64 + l) * 0x7f4a7c15u + 0x2545f491u));
      }
    }
    hash = wave_sum_u32(hs);
    uint64_t cand = __ballot(l < kMemoB && E.memob_key[l < kMemoB ? l : 0] == key && E.memob_hash[l < kMemoB ? l : 0] == hash);
    while (cand) {
      const int e = __builtin_ctzll(cand);
      cand &= cand - 1;
      const CoefMemoBig &m = S->memob[e];
      const uint32_t after = l < kMemoDw ? m.after[l] : 0u;
      const uint64_t f = m.frac;
      bool diff = l < kMemoDw && ((m.before[l] ^ cur_st) & mask);
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (k < nper) diff |= m.coef[k * 64 + l] != cf[k];
      if (__ballot(diff) == 0) {  // a repeat: replay its result
        wsync();
        if (l < kMemoDw) st32[kMemoDw0 + l] = (cur_st & ~mask) | (after & mask);
        if (l == 0) E.cod[E.cur].frac += f;
        wsync();
        return;
      }
    }
    // a miss: the entry takes the levels and the entry states now (no copy held across the walk)
    bslot = E.memob_next;
    CoefMemoBig &m = S->memob[bslot];
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (k < nper) m.coef[k * 64 + l] = cf[k];
    if (l < kMemoDw) m.before[l] = cur_st;
    if (l == 0) m.key = 0;
    wsync();
    E.memob_key[bslot] = 0;  // invalid until its count is in
    wsync();
  }
  HM_T0(t_stage);
  const int n = d.width * d.width;
  const uint16_t *scan = kScan[d.scan_type] + scan_base(ilog2(d.width) - 2);
  const bool staged = n <= 256;
  int16_t *ls = E.u.cs.lev;
  const cab::ScanTables tab(d);
  if (lid() < (n >> 4)) E.u.cs.cg[lid()] = tab.scan_cg[lid()];
  if (memo_on) {
    // 4x4 / 8x8: every level is already in cur_cf (two per lane, raster order): staged by a lane
    // shuffle instead of a second read of the coefficients from the chain state
    const int r = l < n ? scan[l] : 0;
    const uint32_t v = (uint32_t)__shfl((int)cur_cf, r >> 1, HVX_WAVE);
    if (l < n) {
      ls[l] = (int16_t)(r & 1 ? v >> 16 : v & 0xffffu);
      E.u.cs.ras[l] = (int16_t)r;
      int sc = 0;
#pragma unroll
      for (int pat = 0; pat < 4; pat++) sc |= cab::sig_ctx(pat, tab.first_sig, tab.single, r, tab.lw, tab.ch) << (6 * pat);
      E.u.cs.sig[l] = sc;
    }
  } else if (staged) {
    for (int i = lid(); i < n; i += 64) {
      const int r = scan[i];
      ls[i] = coef[r];
      E.u.cs.ras[i] = (int16_t)r;
      int sc = 0;
#pragma unroll
      for (int pat = 0; pat < 4; pat++) sc |= cab::sig_ctx(pat, tab.first_sig, tab.single, r, tab.lw, tab.ch) << (6 * pat);
      E.u.cs.sig[i] = sc;
    }
  } else {
    for (int i = lid(); i < n; i += 64) ls[i] = coef[scan[i]];
  }
  CoderLane L{E.cod[E.cur].st, 0};
  wsync();
  HM_TADD(PR_COEF_STAGE, t_stage);
  HM_T0(t_walk);
  const StagedScan env{E.u.cs.cg, E.u.cs.ras, E.u.cs.sig, scan, tab.first_sig, tab.single, !staged};
  // the mask-driven walk for every size (a third walk instance in this function measured 20%
  // slower overall: register pressure)
  coeff_count_staged(d, env, ls, L);
  E.cod[E.cur].frac += L.frac;
  wsync();
  HM_TADD(PR_COEF_WALK, t_walk);
  HM_TADD(PR_COEF4 + ilog2(d.width) - 2, t_desc);
  if (memo_on) {  // remember the count (FIFO slot)
    const int slot = E.memo_next;
    CoefMemo &m = S->memo[slot];
    const uint32_t *st32 = reinterpret_cast<const uint32_t *>(E.cod[E.cur].st);
    if (l < kMemoDw) { m.before[l] = cur_st; m.after[l] = st32[kMemoDw0 + l]; }
    if (l < d.width * d.width / 2) m.coef[l] = cur_cf;
    const int nx = slot + 1 == kMemoK ? 0 : slot + 1;
    if (l == 0) { m.key = key; m.hash = hash; m.frac = L.frac; S->memo_next = nx; }
    wsync();
    E.memo_key[slot] = key;
    E.memo_hash[slot] = hash;
    E.memo_next = nx;
    wsync();
  }
  if (bslot >= 0) {  // the 16x16 / 32x32 entry's count
    CoefMemoBig &m = S->memob[bslot];
    const uint32_t *st32 = reinterpret_cast<const uint32_t *>(E.cod[E.cur].st);
    if (l < kMemoDw) m.after[l] = st32[kMemoDw0 + l];
    const int nx = bslot + 1 == kMemoB ? 0 : bslot + 1;
    if (l == 0) { m.key = key; m.hash = hash; m.frac = L.frac; S->memob_next = nx; }
    wsync();
    E.memob_key[bslot] = key;
    E.memob_hash[bslot] = hash;
    E.memob_next = nx;
    wsync();
  }
}
// TEncEntropy::estimateBit (TEncEntropy.cpp:685) from the current coder
// The entries TEncSbac::estBit writes (exactly those of estbit_update), one per lane: two
// rounds of 64 entries instead of ~200 serial table reads by the whole wave.
// The call overwrites a fixed set of entries with values that depend only on (w, h, ch) and the
// context states 28 .. 179, so a call whose inputs equal the previous call's leaves the table as
// it is (the RQT's transform-skip pass re-estimates from the state its first pass loaded, and the
// intra searches re-estimate from restored states): such a call returns after one compare.
__device__ void estimate_bit(int w, int h, int ch) {
  HM_PROF(PR_EST);
  const uint8_t *st = E.cod[E.cur].st;
  hvx_estbits *e = &E.est;
#define EB(ctx, v) (int32_t)ebits(st[(ctx)] ^ (v))
  const int l = lid(), b = l & 1;
  static_assert(HVX_CTX_QT_CBF >= 28 && HVX_CTX_ABS + 6 <= 180, "estBit's context range");
  {
    const uint32_t key = (uint32_t)(w | h << 8 | ch << 16) + 1;
    const uint32_t cur = l < 38 ? reinterpret_cast<const uint32_t *>(st)[7 + l] : 0;
    const bool same = __ballot(l < 38 && cur != E.est_st[l]) == 0;
    if (E.est_key == key && same) return;
    if (l < 38) E.est_st[l] = cur;
    if (l == 0) E.est_key = key;
  }
  // round 1: cbf (20), root cbf (8), sig CG (4), significance (<= 28)
  if (l < 20) e->blockCbpBits[l >> 1][b] = EB(HVX_CTX_QT_CBF + (l >> 1), b);
  else if (l < 28) e->blockRootCbpBits[(l - 20) >> 1][b] = EB(HVX_CTX_QT_ROOT_CBF + ((l - 20) >> 1), b);
  else if (l < 32) e->significantCoeffGroupBits[(l - 28) >> 1][b] = EB(HVX_CTX_SIG_CG + ch * 2 + ((l - 28) >> 1), b);
  else {
    const int type = (w == 4 && h == 4) ? 0 : (w == 8 && h == 8) ? 1 : 2;
    const int first = estbit_sig_start(ch, type), num = estbit_sig_size(ch, type), off = ch ? 28 : 0;
    const int single = estbit_sig_start(ch, 3);
    // the index list: [0 if first > 0], single, first .. first + num - 1
    const int lead = first > 0 ? 2 : 1, k = (l - 32) >> 1;
    int idx = -1;
    if (k < lead + num) idx = (first > 0 && k == 0) ? 0 : (k == lead - 1) ? single : first + (k - lead);
    if (idx >= 0) e->significantBits[off + idx][b] = EB(HVX_CTX_SIG + off + idx, b);
  }
  // round 2: greater-1 (<= 32), level-abs (<= 8), last X / Y prefixes (<= 11 each), rice (4)
  if (l < 32) {
    const int i = l >> 1;
    if (i < (ch ? 8 : 16)) e->greaterOneBits[(ch ? 16 : 0) + i][b] = EB(HVX_CTX_ONE + (ch ? 16 : 0) + i, b);
  } else if (l < 40) {
    const int i = (l - 32) >> 1;
    if (i < (ch ? 2 : 4)) e->levelAbsBits[(ch ? 4 : 0) + i][b] = EB(HVX_CTX_ABS + (ch ? 4 : 0) + i, b);
  } else if (l < 62) {
    const int yax = l >= 51, c = l - (yax ? 51 : 40);
    const int n = yax ? h : w, cl = estbit_log2(n) - 2;
    const int o = ch ? 0 : cl * 3 + ((cl + 1) >> 2), sft = ch ? cl : (cl + 3) >> 2;
    const int base = (yax ? HVX_CTX_LAST_Y : HVX_CTX_LAST_X) + ch * 15 + o;
    const int G = estbit_group_idx(n - 1);
    if (c <= G) {
      int bits = 0;
      for (int q = 0; q < c; q++) bits += EB(base + (q >> sft), 1);
      if (c < G) bits += EB(base + (c >> sft), 0);
      if (yax) e->lastYBits[ch][c] = bits;
      else e->lastXBits[ch][c] = bits;
    }
  } else {
    e->golombRiceAdaptationStatistics[l - 62] = 0;
    e->golombRiceAdaptationStatistics[l - 60] = 0;
  }
#undef EB
  wsync();
}

// ============================================================================================
// xEncodeTransform (TEncEntropy.cpp:200) and encodeCoeff (:615)
// ============================================================================================
template <int LV>
__device__ void encode_transform(const Cu *cu, const Tu &t) {
  const int rel = tu_abs_rel(t);
  const int trd = tu_depth_rel(t);
  const int subdiv = cu->p[rel].tr_idx > trd;
  const int l2 = t.log2;
  int cbf0 = cbf_at(&cu->p[rel], 0, trd), cbf1 = cbf_at(&cu->p[rel], 1, trd), cbf2 = cbf_at(&cu->p[rel], 2, trd);
  const int any = cbf0 | cbf1 | cbf2;
  const int intra = cu->p[rel].pred == MODE_INTRA;
  if (intra && cu->p[rel].part == SIZE_NxN && trd == 0) {
  } else if (l2 > 5) {
  } else if (l2 == 2) {
  } else if (l2 == qt_min_log2(cu, rel)) {
  } else code_subdiv(subdiv, 5 - l2);
  const int first = trd == 0;
  for (int c = 1; c < 3; c++)
    if (first || t.all[c])
      if (first || cbf_at(&cu->p[rel], c, trd - 1)) code_qt_cbf(cu, t, c, !subdiv);
  if (subdiv) {
    if constexpr (LV < 3) {
      TU_LOCAL(ch);
      tu_child(ch, t, 1);
      do encode_transform<LV + 1>(cu, ch); while (tu_next(ch, t));
    } else HMC(false, 21, LV, 0);
    return;
  }
  if (!intra && trd == 0 && !cbf_at(&cu->p[rel], 1, 0) && !cbf_at(&cu->p[rel], 2, 0)) {
  } else code_qt_cbf(cu, t, 0, 1);
  if (any)
    for (int c = 0; c < 3; c++) {
      const int cb = c == 0 ? cbf0 : c == 1 ? cbf1 : cbf2;
      if (tu_proc(t, c) && cb) code_coeff_nxn(cu, t, c, cu->coef + coff(c) + t.off[c]);
    }
}
__device__ void encode_coeff(const Cu *cu, int rel) {
  if (cu->p[rel].pred != MODE_INTRA) {
    if (!(cu->p[rel].merge && cu->p[rel].part == SIZE_2Nx2N)) cbin(X_ROOT_CBF, cu_qt_root_cbf(cu, rel));
    if (!cu_qt_root_cbf(cu, rel)) return;
  }
  TU_LOCAL(t);
  tu_root(t, cu, 0);
  encode_transform<0>(cu, t);
}

// ============================================================================================
// Samples: originals, the reconstruction (picture + the current CTU's window), yuv ops
// ============================================================================================
__device__ void copy_org_to_yuv(Yuv *dst, const Cu *cu) {
  const int w = cu->width, cx = cu->x, cy = cu->y;
  for (int c = 0; c < 3; c++) {
    const int s = c ? 1 : 0, n = w >> s, x0 = cx >> s, y0 = cy >> s, W = E.P.w >> s, H = E.P.h >> s;
    const uint8_t *org = E.P.org[c];
    const int os = E.P.org_stride[s];
    int16_t *d = yaddr(dst, c, 0, 0);
    const int ds = ystride(c), sh = ilog2(n);
    for (int i = lid(); i < n * n; i += 64) {
      const int y = i >> sh, x = i & (n - 1), px = x0 + x, py = y0 + y;
      d[y * ds + x] = (px < W && py < H) ? org[py * os + px] : 0;
    }
  }
  wsync();
}
// a sample of the picture reconstruction (the CTU being decided reads its own window)
__device__ __forceinline__ int rec_px(int c, int x, int y) {
  const int s = c ? 1 : 0, cs = 64 >> s;
  const int wx = x - E.ctu_x * cs, wy = y - E.ctu_y * cs;
  if ((unsigned)wx < (unsigned)cs && (unsigned)wy < (unsigned)cs) return E.S->win[coff(c) + wy * cs + wx];
  HMC(x >= 0 && y >= 0 && x < (E.P.w >> s) && y < (E.P.h >> s), 3, x, y + 1000 * c);
  if (HM_CHECKING && !(x >= 0 && y >= 0 && x < (E.P.w >> s) && y < (E.P.h >> s))) return 0;
  return E.P.rec[c][y * E.P.rec_stride[s] + x];
}
// writes of the reconstruction inside the current CTU (TComPicYuv rec), CU/TU-relative
__device__ __forceinline__ uint8_t *win_at(int c, int x, int y) {  // picture coordinates of component c
  const int s = c ? 1 : 0, cs = 64 >> s;
  HMC((unsigned)(x - E.ctu_x * cs) < (unsigned)cs && (unsigned)(y - E.ctu_y * cs) < (unsigned)cs, 4, x, y + 1000 * c);
  if (HM_CHECKING && !((unsigned)(x - E.ctu_x * cs) < (unsigned)cs && (unsigned)(y - E.ctu_y * cs) < (unsigned)cs)) return &E.S->win[0];
  return &E.S->win[coff(c) + (y - E.ctu_y * cs) * cs + (x - E.ctu_x * cs)];
}
// xCopyYuv2Pic (TEncCu.cpp:1514)
__device__ void yuv_to_pic_comp(Yuv *src, const Cu *cu, int c) {
  const int s = c ? 1 : 0, n = cu->width >> s, x0 = cu->x >> s, y0 = cu->y >> s;
  const int W = E.P.w >> s, H = E.P.h >> s, sh = ilog2(n);
  const int16_t *p = yaddr(src, c, 0, 0);
  for (int i = lid(); i < n * n; i += 64) {
    const int y = i >> sh, x = i & (n - 1);
    if (x0 + x < W + 8 && y0 + y < H + 8) *win_at(c, x0 + x, y0 + y) = (uint8_t)p[y * ystride(c) + x];
  }
  wsync();
}
__device__ void yuv_to_pic(Yuv *src, const Cu *cu) {
  for (int c = 0; c < 3; c++) yuv_to_pic_comp(src, cu, c);
}
// xCopyYuv2Tmp (:1541)
__device__ void yuv_child_to_parent(Yuv *dst, Yuv *src, int idx, int child_w) {
  for (int c = 0; c < 3; c++) {
    const int s = c ? 1 : 0, n = child_w >> s, ox = (idx & 1) * n, oy = (idx >> 1) * n, sh = ilog2(n);
    for (int i = lid(); i < n * n; i += 64) {
      const int y = i >> sh, x = i & (n - 1);
      *yaddr_w(dst, c, ox + x, oy + y, 2 * child_w) = *yaddr_w(src, c, x, y, child_w);
    }
  }
  wsync();
}
enum { YOP_SUB, YOP_ADD_CLIP, YOP_COPY, YOP_CLEAR };
__device__ void yuv_op(int op, Yuv *dst, Yuv *a, Yuv *b, int w) {
  for (int c = 0; c < 3; c++) {
    const int n = c ? w >> 1 : w, s = ystride(c), sh = ilog2(n);
    int16_t *d = yaddr(dst, c, 0, 0);
    const int16_t *pa = a ? yaddr(a, c, 0, 0) : nullptr, *pb = b ? yaddr(b, c, 0, 0) : nullptr;
    for (int i = lid(); i < n * n; i += 64) {
      const int k = (i >> sh) * s + (i & (n - 1));
      int v;
      if (op == YOP_SUB) v = pa[k] - pb[k];
      else if (op == YOP_ADD_CLIP) v = clip_pel(pa[k] + pb[k]);
      else if (op == YOP_COPY) v = pa[k];
      else v = 0;
      d[k] = (int16_t)v;
    }
  }
  wsync();
}

// ============================================================================================
// TComRdCost: calcRdCost (TComRdCost.cpp:57), the DF_SAD variant, getCost, getDistPart
// ============================================================================================
__device__ __forceinline__ double rd_cost(uint32_t bits, uint32_t dist) {
  return floor(__dadd_rn(__dadd_rn((double)dist, __dmul_rn((double)bits, E.P.lambda)), 0.5));
}
__device__ __forceinline__ double rd_cost_sad(uint32_t bits, uint32_t dist) {
  return floor(__dadd_rn((double)dist, floor(__dadd_rn(__dmul_rn((double)bits, (double)E.P.lambda_motion), 0.5)) / 65536.0));
}
__device__ __forceinline__ uint32_t mv_cost_bits(uint32_t bits) { return (uint32_t)(E.P.lambda_motion * bits) >> 16; }
// The SSIM cost of TEncCu's comparisons (HVX_RD_SSIM, include/hvx_types.h; restated by cu_dssim /
// cu_cost in oracle/hvx_oracle_cu.c): one window per block, compute_SSIM's float order
// (stvssim.c:491-566) and its [1, 1.01) clamp
__device__ __forceinline__ float ssim_block16(const int16_t *o, const int16_t *r, int stride, int wint) {
  const float C1 = 0.01f * 0.01f * (float)(255 * 255), C2 = 0.03f * 0.03f * (float)(255 * 255);
  const float wgt = 1.0f / (float)(wint * wint);
  float mo = 0, me = 0, vo = 0, ve = 0, cov = 0;
  for (int n = 0; n < wint; n++)
    for (int m = 0; m < wint; m++) {
      const int po = o[n * stride + m], pe = r[n * stride + m];
      mo += wgt * po; me += wgt * pe;
      vo += wgt * po * po; ve += wgt * pe * pe; cov += wgt * po * pe;
    }
  const float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cov - mo * me);
  float v = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
  v /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
  if (v >= 1.0 && v < 1.01) v = 1.0f;
  return v;
}
// D of a CU: its 8x8 luma blocks, then 4x4 Cb, Cr blocks, one block per lane; the terms / 4 summed
// in that order in double (blocks outside the picture skipped)
__device__ __noinline__ double cu_dssim(const Cu *cu, Yuv *org, Yuv *reco) {
  const int n = cu->width >> 3, nb = n * n, total = 3 * nb;
  const int cx = cu->x, cy = cu->y;
  for (int k = lid(); k < total; k += 64) {
    const int c = k / nb, i = k - c * nb, by = i / n, bx = i - by * n;
    const int sh = c ? 1 : 0, b = c ? 4 : 8;
    const bool in = (cx >> sh) + bx * b < (E.P.w >> sh) && (cy >> sh) + by * b < (E.P.h >> sh);
    E.ssim_t[k] = in ? 1.0f - ssim_block16(yaddr(org, c, bx * b, by * b), yaddr(reco, c, bx * b, by * b), ystride(c), b) : -1.0f;
  }
  wsync();
  double d = 0;
  for (int k = 0; k < total; k++) {
    const float t = E.ssim_t[k];
    if (t >= 0.0f) d += 0.25 * (double)t;
  }
  wsync();
  return d;
}
// compute_stVSSIM's directional weights for `used` frames (stvssim.c:615-640)
__device__ __forceinline__ void stv_weights(int wint, int used, float *wgta, float *wgtb) {
  const float wa = 0.6f, wb = 1.0f - wa;
  if (wint == 4) {
    wgta[0] = wgta[2] = wgta[1] = wgta[3] = wa / (wint * (used));
    wgtb[0] = wgtb[2] = wgtb[1] = wgtb[3] = wb / ((wint * wint - wint) * (used));
  } else {
    wgta[0] = wgta[2] = wa / (3 * wint * (used));
    wgta[1] = wgta[3] = wa / ((3 * wint - 2) * (used));
    wgtb[0] = wgtb[2] = wb / ((wint * wint - 3 * wint) * (used));
    wgtb[1] = wgtb[3] = wb / ((wint * wint - 3 * wint + 2) * (used));
  }
}
// the history frames' terms of one window's 4 x 5 directional sums (:665-699 for o < used - 1),
// added to acc[k * 5 + {mo, me, vo, ve, cov}]: every accumulator receives its terms in the
// reference's (o, n, m) order.  hist[6o + hc] / hist[6o + 3 + hc]: original / reconstruction plane
__device__ __forceinline__ void stv_hist_acc(const uint8_t *const *hist, int n_hist, int hc, int hs, int wint, int px,
                                             int py, const float *wgta, const float *wgtb, float *acc) {
  for (int o = 0; o < n_hist; o++) {
    const uint8_t *ho = hist[6 * o + hc] + (size_t)py * hs + px;
    const uint8_t *hr = hist[6 * o + 3 + hc] + (size_t)py * hs + px;
    for (int n = 0; n < wint; n++)
      for (int m = 0; m < wint; m++) {
        const int po = ho[n * hs + m], pe = hr[n * hs + m];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const float wgt = orient_weight(k, wint, n, m, wgta[k], wgtb[k]);
          acc[k * 5 + 0] += wgt * po; acc[k * 5 + 1] += wgt * pe;
          acc[k * 5 + 2] += wgt * po * po; acc[k * 5 + 3] += wgt * pe * pe; acc[k * 5 + 4] += wgt * po * pe;
        }
      }
  }
}
// the window's record in hvx_hm_picture.stv_sums (include/hvx.h hvx_hm_stv_prepare): c 0 luma 8x8, else
// chroma 8x8 / 4x4 (wint), origin (px, py) on the 4-sample grid of the component
__device__ __forceinline__ size_t stv_sums_window(int c, int wint, int px, int py, int w, int h) {
  const int nx0 = (w - 8) / 4 + 1, ny0 = (h - 8) / 4 + 1;
  if (c == 0) return (size_t)(py >> 2) * nx0 + (px >> 2);
  const int nx1 = ((w >> 1) - 8) / 4 + 1, ny1 = ((h >> 1) - 8) / 4 + 1, nx2 = ((w >> 1) - 4) / 4 + 1;
  if (wint == 8) return (size_t)ny0 * nx0 + (size_t)(py >> 2) * nx1 + (px >> 2);
  return (size_t)ny0 * nx0 + (size_t)ny1 * nx1 + (size_t)(py >> 2) * nx2 + (px >> 2);
}
// The stVSSIM cost (HVX_RD_STVSSIM, include/hvx_types.h hvx_hm_picture.hist; restated by cu_dstv in
// oracle/hvx_oracle_cu.c): distortionstVSSIM (stvssim.c:831-855) per 16x16 luma area of the CU.
// One lane per window (compute_stVSSIM's loop body :655-811 in its float order): the four directional
// 3-D SSIMs over the history frames (most recent first: from the picture's precomputed stv_sums, or
// summed here) and then the CU's own original / reconstruction, the direction vote of calOrit (:336)
// on the map, and the plain SSIM of the current frame; the window's ssim * ssim3d goes to E.ssim_t,
// averaged per block in window order.
__device__ float stv_window(int c, int wint, int lx, int ly, int px, int py, const int16_t *org, const int16_t *rec,
                            int ystr) {
  const int used = E.P.hist_n + 1, hc = c == 2 ? 1 : c, uv = c ? 2 : 1;
  float wgta[4], wgtb[4];
  stv_weights(wint, used, wgta, wgtb);
  const float C1 = 0.01f * 0.01f * (float)(255 * 255), C2 = 0.03f * 0.03f * (float)(255 * 255);
  float acc[20];
  if (E.P.stv_sums) {
    const float *t = E.P.stv_sums + 20 * stv_sums_window(c, wint, px, py, E.P.w, E.P.h);
#pragma unroll
    for (int i = 0; i < 20; i++) acc[i] = t[i];
  } else {
#pragma unroll
    for (int i = 0; i < 20; i++) acc[i] = 0.0f;
    stv_hist_acc(E.P.hist, E.P.hist_n, hc, E.P.hist_stride[c ? 1 : 0], wint, px, py, wgta, wgtb, acc);
  }
  for (int n = 0; n < wint; n++)  // o = used - 1: the current picture
    for (int m = 0; m < wint; m++) {
      const int po = org[(ly + n) * ystr + lx + m], pe = rec[(ly + n) * ystr + lx + m];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const float wgt = orient_weight(k, wint, n, m, wgta[k], wgtb[k]);
        acc[k * 5 + 0] += wgt * po; acc[k * 5 + 1] += wgt * pe;
        acc[k * 5 + 2] += wgt * po * po; acc[k * 5 + 3] += wgt * pe * pe; acc[k * 5 + 4] += wgt * po * pe;
      }
    }
  float s3[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const float mo = acc[k * 5], me = acc[k * 5 + 1], vo = acc[k * 5 + 2], ve = acc[k * 5 + 3], cv = acc[k * 5 + 4];
    const float varo = fabsf(vo - mo * mo), vare = fabsf(ve - me * me), covo = fabsf(cv - mo * me);
    float v = (float)((2.0 * mo * me + C1) * (2.0 * covo + C2));
    v /= (float)(mo * mo + me * me + C1) * (varo + vare + C2);
    s3[k] = v;
    if (s3[k] >= 1.0 && s3[k] < 1.01) s3[k] = 1.0f;
  }
  // calOrit over the window's samples (the map is per 4x4 luma block; chroma reads luma coordinates)
  const float kOrient[4] = {0, 3.1415926f / 4, 3.1415926f / 2, 3.1415926f * 3 / 4};
  short orit[4] = {0, 0, 0, 0};
  for (int n = 0; n < wint; n++)
    for (int m = 0; m < wint; m++) {
      const float od = E.P.dirs ? E.P.dirs[(((py + n) * uv) >> 2) * E.P.dirs_stride + (((px + m) * uv) >> 2)] : 0.0f;
      float dn[4], dx = 10000.0f;
      for (int q = 0; q < 4; q++) { dn[q] = (float)fabs(od - kOrient[q]); if (dn[q] < dx) dx = dn[q]; }
      for (int q = 0; q < 4; q++) if (fabs(dx - dn[q]) < 0.01f) orit[q]++;
    }
  short tmp = 0, inx = 0;
  for (int q = 0; q < 4; q++) if (orit[q] > tmp) { tmp = orit[q]; inx = (short)q; }
  int q;
  for (q = 0; q < 4; ++q) if ((tmp - orit[q]) < 10 && inx != q) break;
  const float t3 = q == 4 ? s3[inx] : (s3[inx] + s3[q]) / 2;
  // the plain SSIM of the current frame (:758-807), no clamp
  const float wgt = 1.0f / (wint * wint);
  float a = 0, b = 0, va = 0, vb = 0, cab = 0;
  for (int n = 0; n < wint; n++)
    for (int m = 0; m < wint; m++) {
      const int po = org[(ly + n) * ystr + lx + m], pe = rec[(ly + n) * ystr + lx + m];
      a += wgt * po; b += wgt * pe;
      va += wgt * po * po; vb += wgt * pe * pe; cab += wgt * po * pe;
    }
  const float varo = fabsf(va - a * a), vare = fabsf(vb - b * b), covo = fabsf(cab - a * b);
  float ts = (float)((2.0 * a * b + C1) * (2.0 * covo + C2));
  ts /= (float)(a * a + b * b + C1) * (varo + vare + C2);
  return ts * t3;
}
// stvssimx of one block from its window terms (:817-824) -> 1 - stVSSIM (distortionstVSSIM :840)
__device__ __forceinline__ float stv_block(const float *t, int nw) {
  float x = 0;
  for (int k = 0; k < nw; k++) x += t[k];
  x /= (float)nw;
  if (x >= 1.0 && x < 1.01) x = 1.0f;
  return 1.0f - x;
}
// D of a CU: tasks = per 16x16 area (raster) its 9 luma windows then the Cb and Cr window; an 8x8
// CU: one luma, one Cb, one Cr window (4x4 chroma), weighted 1/4
__device__ __noinline__ double cu_dstv(const Cu *cu, Yuv *org, Yuv *reco) {
  const bool small = cu->width == 8;
  const int n = small ? 1 : cu->width >> 4, per = small ? 3 : 11, total = n * n * per;
  for (int k = lid(); k < total; k += 64) {
    const int mb = k / per, w = k - mb * per, my = mb / n, mx = mb - my * n;
    int c, wint, lx, ly;
    if (small) {
      c = w; wint = c ? 4 : 8; lx = 0; ly = 0;
    } else if (w < 9) {
      c = 0; wint = 8; lx = 16 * mx + 4 * (w % 3); ly = 16 * my + 4 * (w / 3);
    } else {
      c = w - 8; wint = 8; lx = 8 * mx; ly = 8 * my;
    }
    const int sh = c ? 1 : 0;
    const bool in = cu->x + 16 * mx < E.P.w && cu->y + 16 * my < E.P.h;
    E.ssim_t[k] = in ? stv_window(c, wint, lx, ly, (cu->x >> sh) + lx, (cu->y >> sh) + ly, yaddr(org, c, 0, 0),
                                  yaddr(reco, c, 0, 0), ystride(c))
                     : 0.0f;
  }
  wsync();
  double d = 0;
  for (int mb = 0; mb < n * n; mb++) {
    const int my = mb / n, mx = mb - my * n;
    if (cu->x + 16 * mx >= E.P.w || cu->y + 16 * my >= E.P.h) continue;
    const float *t = E.ssim_t + mb * per;
    const float dy = stv_block(t, small ? 1 : 9), du = stv_block(t + (small ? 1 : 9), 1), dv = stv_block(t + (small ? 2 : 10), 1);
    const double dm = (double)dy * 1.0 + (double)du * 1.0 + (double)dv * 1.0;
    d += small ? 0.25 * dm : dm;
  }
  wsync();
  return d;
}
// the cost TEncCu compares: calcRdCost(bits, dist), or the SSIM / stVSSIM cost (dssim already measured)
__device__ __forceinline__ double cu_cost(double dssim, uint32_t bits, uint32_t dist) {
  if (E.P.rd_metric == HVX_RD_SSE) return rd_cost(bits, dist);
  return dssim + E.P.lambda_ssim * ((double)bits > 0.5 ? (double)bits : 0.5);
}
// the SSIM measurements stay out of line: the SSE decision (the headline) keeps its callers' code
__device__ __forceinline__ double measure_ssim(Cu *cu, Yuv *org, Yuv *reco) {
  if (__builtin_expect(E.P.rd_metric == HVX_RD_SSE, 1)) return 0.0;
  const double d = E.P.rd_metric == HVX_RD_STVSSIM ? cu_dstv(cu, org, reco) : cu_dssim(cu, org, reco);
  cu->dssim = d;
  wsync();
  return d;
}
__device__ uint32_t sse_wave(const int16_t *a, int sa, const int16_t *b, int sb, int w, int h) {
  HM_PROF(PR_DIST);
  uint32_t s = 0;
  const int n = w * h, sh = ilog2(w);
  for (int i = lid(); i < n; i += 64) {
    const int y = i >> sh, x = i & (w - 1);
    const int d = (b ? (int)b[y * sb + x] : 0) - (int)a[y * sa + x];
    s += (uint32_t)(d * d);
  }
  return wave_sum_u32(s);
}
__device__ __forceinline__ uint32_t weigh(uint32_t sse, int comp) {
  if (comp) return (uint32_t)__dmul_rn(E.P.chroma_weight[comp - 1], (double)sse);
  return sse;
}
__device__ uint32_t dist_part(const int16_t *a, int sa, const int16_t *b, int sb, int w, int h, int comp) {
  return weigh(sse_wave(a, sa, b, sb, w, h), comp);
}
__device__ uint32_t yuv_dist(Yuv *a, Yuv *b, int w) {
  uint32_t d = 0;
  for (int c = 0; c < 3; c++) {
    const int n = c ? w >> 1 : w;
    d += dist_part(yaddr(a, c, 0, 0), ystride(c), yaddr(b, c, 0, 0), ystride(c), n, n, c);
  }
  return d;
}

// ============================================================================================
// Transform / quantisation / RDOQ / inverse through the pinned wave kernels (hvx_tu.hpp)
// ============================================================================================
// the TU pipeline's scratch: LDS up to 16x16, the chain state for 32x32
template <int L>
__device__ __forceinline__ TuSmem<L> &tu_smem() {
  if constexpr (L == 3) return E.S->tu3;
  else return *reinterpret_cast<TuSmem<L> *>(&E.u);
}
template <int L>
__device__ int32_t tu_fwd_l(const hvx_tu_desc &d, const int16_t *resi, int rs, int16_t *coef) {
  HM_PROF(PR_TUF);
#if defined(HM_PROFILE) && !defined(HM_PROF_WALK) && !defined(HVX_RDOQ_PROF_SUB) && !defined(HM_PROF_RQT)
  ProfScope prof_size_(12 + L);
#endif
  TuSmem<L> &s = tu_smem<L>();
  constexpr int N = 4 << L;
  HM_T0(t_in);
  const uint16_t *scan_g = kScan[d.scan_type] + scan_base(L);
  for (int i = lid(); i < N * N; i += 64) {
    s.a[i] = resi[(i >> (L + 2)) * rs + (i & (N - 1))];
    if constexpr (L < 3) E.scan[i] = scan_g[i];
  }
  if constexpr (L < 3)
    if (lid() < (N * N >> 4)) E.scan_cg[lid()] = kScanCG[d.scan_type][cg_base(L) + lid()];
  wsync();
  HM_TADD(PR_TUF_IN, t_in);
  HM_T0(t_fwd);
  // the RDOQ's serial passes read the staged scan tables (LDS) instead of the constant tables
  const int32_t abs_sum = L < 3 ? tu_forward<L>(s, d, &E.est, nullptr, E.scan, E.scan_cg) : tu_forward<L>(s, d, &E.est, nullptr);
  HM_TADD(PR_TUF_FWD, t_fwd);
  HM_T0(t_out);
  for (int i = lid(); i < N * N; i += 64) coef[i] = (int16_t)s.lev[i];
  wsync();
  HM_TADD(PR_TUF_OUT, t_out);
  return abs_sum;
}
template <int L>
__device__ void tu_inv_l(const hvx_tu_desc &d, const int16_t *coef, int16_t *resi, int rs) {
  HM_PROF(PR_TUI);
  TuSmem<L> &s = tu_smem<L>();
  constexpr int N = 4 << L;
  for (int i = lid(); i < N * N; i += 64) s.lev[i] = coef[i];
  wsync();
  tu_inverse<L>(s, d);
  for (int i = lid(); i < N * N; i += 64) resi[(i >> (L + 2)) * rs + (i & (N - 1))] = (int16_t)s.lev[i];
  wsync();
}
// transformNxN; sets the TU's CBF (TComTrQuant.cpp:1543)
__device__ int32_t transform_tu(Cu *cu, const Tu &t, int comp, const int16_t *resi, int rs, int16_t *coef) {
  tu_desc(cu, t, comp);
  const hvx_tu_desc &d = E.td;
  HMC(d.log2_size >= 2 && d.log2_size <= 5 && t.off[comp] + t.w[comp] * t.h[comp] <= (comp ? 1024 : 4096) &&
          tu_abs_rel(t) + tu_nparts(t, comp) <= cu->nparts, 10, d.log2_size * 100 + comp, t.off[comp]);
  int32_t abs_sum;
  switch (d.log2_size) {
    case 2: abs_sum = tu_fwd_l<0>(d, resi, rs, coef); break;
    case 3: abs_sum = tu_fwd_l<1>(d, resi, rs, coef); break;
    case 4: abs_sum = tu_fwd_l<2>(d, resi, rs, coef); break;
    default: abs_sum = tu_fwd_l<3>(d, resi, rs, coef); break;
  }
  set_cbf_range(cu, comp, tu_abs_rel(t), tu_nparts(t, comp), (abs_sum > 0 ? 1 : 0) << tu_depth_rel(t));
  return abs_sum;
}
__device__ void inv_transform_tu(const Cu *cu, const Tu &t, int comp, const int16_t *coef, int16_t *resi, int rs,
                                 bool desc_ready = false) {
  if (!desc_ready) tu_desc(cu, t, comp);
  const hvx_tu_desc &d = E.td;
  switch (d.log2_size) {
    case 2: tu_inv_l<0>(d, coef, resi, rs); break;
    case 3: tu_inv_l<1>(d, coef, resi, rs); break;
    case 4: tu_inv_l<2>(d, coef, resi, rs); break;
    default: tu_inv_l<3>(d, coef, resi, rs); break;
  }
}
__device__ void blk_copy(int16_t *dst, int ds, const int16_t *src, int ss, int w, int h) {
  const int sh = ilog2(w);
  for (int i = lid(); i < w * h; i += 64) {
    const int y = i >> sh, x = i & (w - 1);
    dst[y * ds + x] = src ? src[y * ss + x] : 0;
  }
  wsync();
}

// ============================================================================================
// Motion compensation (TComPrediction::motionCompensation :517, one PU) into a yuv buffer
// ============================================================================================
// xPredInterBlk (:668) for one component and list, lane-parallel, dst with stride ds
__device__ void mc_blk(bool luma, const int16_t *plane, int stride, int x, int y, int mvx, int mvy, int w, int h, bool bi,
                       int16_t *dst, int ds) {
  int16_t *tmp = E.S->mc.tmp;
  const int sh = luma ? 2 : 3, n = luma ? 8 : 4;
  const int xf = mvx & ((1 << sh) - 1), yf = mvy & ((1 << sh) - 1);
  const int16_t *ref = plane + (y + (mvy >> sh)) * stride + x + (mvx >> sh);
  const int8_t *cx = luma ? kLumaFilter[xf] : kChromaFilter[xf];
  const int8_t *cy = luma ? kLumaFilter[yf] : kChromaFilter[yf];
  const int half = n / 2 - 1;
#ifdef HM_CHECKS
  {
    const int m = luma ? 80 : 40, W = luma ? E.P.w : E.P.w >> 1, H = luma ? E.P.h : E.P.h >> 1;
    const int x0 = x + (mvx >> sh) - half, y0 = y + (mvy >> sh) - half;
    const bool ok = x0 >= -m && y0 >= -m && x0 + w + n <= W + m && y0 + h + n <= H + m && plane != nullptr;
    HMC(ok, 5, x0 + 10000 * (luma ? 1 : 2), y0);
    if (!ok) {
      for (int k = lid(); k < w * h; k += 64) dst[(k / w) * ds + k % w] = 0;
      wsync();
      return;
    }
  }
#endif
  if (yf == 0) {
    for (int k = lid(); k < w * h; k += 64) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = ref + r * stride + c;
      if (xf == 0) dst[r * ds + c] = (int16_t)mc_copy_first(p[0], !bi);
      else {
        int s = 0;
        for (int t = 0; t < n; t++) s += cx[t] * p[t - half];
        dst[r * ds + c] = (int16_t)mc_fir_out(s, true, !bi);
      }
    }
  } else if (xf == 0) {
    for (int k = lid(); k < w * h; k += 64) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = ref + r * stride + c;
      int s = 0;
      for (int t = 0; t < n; t++) s += cy[t] * p[(t - half) * stride];
      dst[r * ds + c] = (int16_t)mc_fir_out(s, true, !bi);
    }
  } else {
    const int16_t *src = ref - half * stride;
    for (int k = lid(); k < w * (h + n - 1); k += 64) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = src + r * stride + c;
      int s = 0;
      for (int t = 0; t < n; t++) s += cx[t] * p[t - half];
      tmp[k] = (int16_t)mc_fir_out(s, true, false);
    }
    wsync();
    for (int k = lid(); k < w * h; k += 64) {
      const int r = k / w, c = k - r * w;
      const int16_t *p = tmp + (r + half) * w + c;
      int s = 0;
      for (int t = 0; t < n; t++) s += cy[t] * p[(t - half) * w];
      dst[r * ds + c] = (int16_t)mc_fir_out(s, false, !bi);
    }
  }
  wsync();
}
__device__ __forceinline__ void clip_mv(const Cu *cu, int &mx, int &my) {  // TComDataCU::clipMv
  const int hmax = (E.P.w + 8 - cu->x - 1) << 2, hmin = (-64 - 8 - cu->x + 1) << 2;
  const int vmax = (E.P.h + 8 - cu->y - 1) << 2, vmin = (-64 - 8 - cu->y + 1) << 2;
  mx = (int16_t)(mx < hmin ? hmin : mx > hmax ? hmax : mx);
  my = (int16_t)(my < vmin ? vmin : my > vmax ? vmax : my);
}
__device__ void mc_pu(const Cu *cu, int ps, int pu, Yuv *dst) {
  HM_PROF(PR_MC);
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, a, w, h);
  part_position(cu, ps, pu, xp, yp, w, h);
  const Part &p = cu->p[a];
  const int r0 = p.ref[0], r1 = p.ref[1];
  const bool v0 = r0 >= 0, v1 = r1 >= 0;
  int mx[2] = {p.mv[0][0], p.mv[1][0]}, my[2] = {p.mv[0][1], p.mv[1][1]};
  const int poc0 = v0 ? E.P.ref_poc[0][r0] : 0, poc1 = v1 ? E.P.ref_poc[1][r1] : 0;
  const bool identical = E.P.slice_type == B_SLICE && v0 && v1 && poc0 == poc1 && mx[0] == mx[1] && my[0] == my[1];
  const bool bi = v0 && v1 && !identical;
  const int l0 = v0 ? 0 : 1;
  clip_mv(cu, mx[0], my[0]);
  clip_mv(cu, mx[1], my[1]);
  const int pl0 = v0 ? E.P.ref_plane[0][r0] : 0, pl1 = v1 ? E.P.ref_plane[1][r1] : 0;
  const int rx = xp - cu->x, ry = yp - cu->y;
  for (int comp = 0; comp < 3; comp++) {
    const bool luma = comp == 0;
    const int cw = luma ? w : w >> 1, chh = luma ? h : h >> 1;
    const int x = luma ? xp : xp >> 1, y = luma ? yp : yp >> 1;
    const int stride = E.P.ref16_stride[luma ? 0 : 1];
    int16_t *o = yaddr(dst, comp, luma ? rx : rx >> 1, luma ? ry : ry >> 1);
    const int os = ystride(comp);
    if (bi) {
      mc_blk(luma, E.P.ref16[pl0][comp], stride, x, y, mx[0], my[0], cw, chh, true, E.S->mc.pr[0], cw);
      mc_blk(luma, E.P.ref16[pl1][comp], stride, x, y, mx[1], my[1], cw, chh, true, E.S->mc.pr[1], cw);
      for (int k = lid(); k < cw * chh; k += 64) {
        const int r = k / cw, c = k - r * cw;
        o[r * os + c] = (int16_t)clip_pel((E.S->mc.pr[0][k] + E.S->mc.pr[1][k] + 16448) >> 7);
      }
      wsync();
    } else {
      const int pl = l0 ? pl1 : pl0;
      mc_blk(luma, E.P.ref16[pl][comp], stride, x, y, mx[l0], my[l0], cw, chh, false, o, os);
    }
  }
}
// motionCompensation(pcCU, m_acYuvPred[list], list, pu): uni prediction of one list; only its
// luma is read (removeHighFreq's other-list prediction of the bi search)
__device__ void mc_pu_list_luma(const Cu *cu, int ps, int pu, int list, int16_t *dst64) {
  HM_PROF(PR_MC);
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, a, w, h);
  part_position(cu, ps, pu, xp, yp, w, h);
  const Part &p = cu->p[a];
  int mx = p.mv[list][0], my = p.mv[list][1];
  clip_mv(cu, mx, my);
  const int pl = E.P.ref_plane[list][p.ref[list]];
  mc_blk(true, E.P.ref16[pl][0], E.P.ref16_stride[0], xp, yp, mx, my, w, h, false, dst64 + (yp - cu->y) * 64 + xp - cu->x, 64);
}
__device__ void mc_cu(const Cu *cu, Yuv *dst) {
  const int ps = cu->p[0].part;
  for (int pu = 0; pu < num_parts_of(ps); pu++) mc_pu(cu, ps, pu, dst);
}

// ============================================================================================
// Merge candidates (getInterMergeCandidates :2182, xGetColMVP :3061, xGetDistScaleFactor :3133)
// ============================================================================================
struct MvField { int16_t mv[2]; int ref; };

__device__ __forceinline__ int dist_scale(int cur_poc, int cur_ref_poc, int col_poc, int col_ref_poc) {
  const int dd = col_poc - col_ref_poc, db = cur_poc - cur_ref_poc;
  if (dd == db) return 4096;
  const int tb = db < -128 ? -128 : db > 127 ? 127 : db, td = dd < -128 ? -128 : dd > 127 ? 127 : dd;
  const int x = (0x4000 + abs(td / 2)) / td;
  const int s = (tb * x + 32) >> 6;
  return s < -4096 ? -4096 : s > 4095 ? 4095 : s;
}
__device__ __forceinline__ int16_t scale_comp(int s, int v) {
  const int r = (s * v + 127 + (s * v < 0)) >> 8;
  return (int16_t)(r < -32768 ? -32768 : r > 32767 ? 32767 : r);
}
__device__ int col_mvp(int list, int ctu, int z, int ref_idx, int16_t *mv) {
  if (!E.P.col_valid) return 0;
  HMC(ctu >= 0 && ctu < E.P.w_ctus * E.P.h_ctus && z >= 0 && z < 256, 7, ctu, z);
  if (HM_CHECKING && !(ctu >= 0 && ctu < E.P.w_ctus * E.P.h_ctus && z >= 0 && z < 256)) return 0;
  const int16_t *f = E.P.col_field + ((size_t)ctu * 16 + (z >> 4)) * 8;
  if (f[0] != MODE_INTER) return 0;
  int cl = E.P.check_ldc ? list : E.P.col_from_l0;
  int cr = f[1 + cl];
  if (cr < 0) {
    cl = 1 - cl;
    cr = f[1 + cl];
    if (cr < 0) return 0;
  }
  const int col_ref_poc = E.P.col_ref_poc[cl][cr];
  const int cmx = f[3 + 2 * cl], cmy = f[4 + 2 * cl];
  const int s = dist_scale(E.P.poc, E.P.ref_poc[list][ref_idx], E.P.col_poc, col_ref_poc);
  if (s == 4096) { mv[0] = (int16_t)cmx; mv[1] = (int16_t)cmy; }
  else { mv[0] = scale_comp(s, cmx); mv[1] = scale_comp(s, cmy); }
  return 1;
}
__device__ void col_positions(const Cu *cu, int ps, int pu, int &br_ctu, int &br_z, int &c_z) {
  const int rb = pu_right_bottom(cu, ps, pu), r = z2r(rb);
  br_ctu = -1;
  br_z = 0;
  if (E.ctu_x * 64 + rpx(r) + 4 < E.P.w && E.ctu_y * 64 + rpy(r) + 4 < E.P.h) {
    if ((r & 15) < 15 && (r >> 4) < 15) { br_z = r2z(r + 17); br_ctu = E.ctu_addr; }
    else if ((r & 15) < 15) { br_z = r2z((r + 17) % 256); }
    else if ((r >> 4) < 15) { br_z = r2z(r + 1); br_ctu = E.ctu_addr + 1; }
    else br_z = 0;
  }
  c_z = pu_center(cu, ps, pu);
}
__device__ __forceinline__ int same_motion(const Part &a, const Part &b) {
  if (a.inter_dir != b.inter_dir) return 0;
  for (int l = 0; l < 2; l++)
    if (a.inter_dir & (1 << l))
      if (a.mv[l][0] != b.mv[l][0] || a.mv[l][1] != b.mv[l][1] || a.ref[l] != b.ref[l]) return 0;
  return 1;
}
__device__ __forceinline__ MvField nb_field(const Nb &n, int list) {
  const Part &q = n.p[n.idx];
  return MvField{{q.mv[list][0], q.mv[list][1]}, q.ref[list]};
}
// the candidate list in LDS-free registers is awkward (dynamic indexing): it lives in the State
struct MergeList { MvField f[10]; int dirs[5]; int is_inter[5]; int n; };

__device__ void merge_candidates(const Cu *cu, int ps, int pu, MergeList &m) {
  const int maxc = E.P.max_merge, isb = E.P.slice_type == B_SLICE;
  for (int i = 0; i < 5; i++) {
    m.f[2 * i] = MvField{{0, 0}, -1};
    m.f[2 * i + 1] = MvField{{0, 0}, -1};
    m.dirs[i] = 0;
    m.is_inter[i] = 0;
  }
  int lt, rt, lb;
  pu_corners(cu, ps, pu, lt, rt, lb);
  int cnt = 0;
  m.n = 0;
  const Nb l = get_pu_left(cu, lb);
  const int a1 = l.valid && !(pu == 1 && (ps == SIZE_Nx2N || ps == SIZE_nLx2N || ps == SIZE_nRx2N)) && nb_inter(l);
  if (a1) {
    m.is_inter[cnt] = 1; m.dirs[cnt] = l.p[l.idx].inter_dir;
    m.f[2 * cnt] = nb_field(l, 0);
    if (isb) m.f[2 * cnt + 1] = nb_field(l, 1);
    cnt++;
  }
  if (cnt == maxc) { m.n = cnt; return; }
  const Nb a = get_pu_above(cu, rt, 0);
  const int b1 = a.valid && !(pu == 1 && (ps == SIZE_2NxN || ps == SIZE_2NxnU || ps == SIZE_2NxnD)) && nb_inter(a);
  if (b1 && (!a1 || !same_motion(l.p[l.idx], a.p[a.idx]))) {
    m.is_inter[cnt] = 1; m.dirs[cnt] = a.p[a.idx].inter_dir;
    m.f[2 * cnt] = nb_field(a, 0);
    if (isb) m.f[2 * cnt + 1] = nb_field(a, 1);
    cnt++;
  }
  if (cnt == maxc) { m.n = cnt; return; }
  const Nb ar = get_pu_above_right(cu, rt, 1);
  const int b0 = nb_inter(ar);
  if (b0 && (!b1 || !same_motion(a.p[a.idx], ar.p[ar.idx]))) {
    m.is_inter[cnt] = 1; m.dirs[cnt] = ar.p[ar.idx].inter_dir;
    m.f[2 * cnt] = nb_field(ar, 0);
    if (isb) m.f[2 * cnt + 1] = nb_field(ar, 1);
    cnt++;
  }
  if (cnt == maxc) { m.n = cnt; return; }
  const Nb bl = get_pu_below_left(cu, lb, 1);
  const int a0 = nb_inter(bl);
  if (a0 && (!a1 || !same_motion(l.p[l.idx], bl.p[bl.idx]))) {
    m.is_inter[cnt] = 1; m.dirs[cnt] = bl.p[bl.idx].inter_dir;
    m.f[2 * cnt] = nb_field(bl, 0);
    if (isb) m.f[2 * cnt + 1] = nb_field(bl, 1);
    cnt++;
  }
  if (cnt == maxc) { m.n = cnt; return; }
  if (cnt < 4) {
    int a_off, w, h;
    part_index_size(cu, ps, pu, a_off, w, h);
    const Nb al = get_pu_above_left(cu, cu->zidx + a_off);
    const int b2 = nb_inter(al);
    if (b2 && (!a1 || !same_motion(l.p[l.idx], al.p[al.idx])) && (!b1 || !same_motion(a.p[a.idx], al.p[al.idx]))) {
      m.is_inter[cnt] = 1; m.dirs[cnt] = al.p[al.idx].inter_dir;
      m.f[2 * cnt] = nb_field(al, 0);
      if (isb) m.f[2 * cnt + 1] = nb_field(al, 1);
      cnt++;
    }
  }
  if (cnt == maxc) { m.n = cnt; return; }
  if (E.P.tmvp) {
    int br_ctu, br_z, c_z, dir = 0;
    col_positions(cu, ps, pu, br_ctu, br_z, c_z);
    int16_t mv[2];
    int ex = br_ctu >= 0 && col_mvp(0, br_ctu, br_z, 0, mv);
    if (!ex) ex = col_mvp(0, E.ctu_addr, c_z, 0, mv);
    if (ex) { dir |= 1; m.f[2 * cnt] = MvField{{mv[0], mv[1]}, 0}; }
    if (isb) {
      ex = br_ctu >= 0 && col_mvp(1, br_ctu, br_z, 0, mv);
      if (!ex) ex = col_mvp(1, E.ctu_addr, c_z, 0, mv);
      if (ex) { dir |= 2; m.f[2 * cnt + 1] = MvField{{mv[0], mv[1]}, 0}; }
    }
    if (dir) { m.dirs[cnt] = dir; m.is_inter[cnt] = 1; cnt++; }
  }
  if (cnt == maxc) { m.n = cnt; return; }
  int arr = cnt;
  const int cutoff = arr;
  if (isb) {
    const int l0[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3}, l1[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};
    for (int idx = 0; idx < cutoff * (cutoff - 1) && arr != maxc; idx++) {
      const int i = l0[idx], j = l1[idx];
      if (m.is_inter[i] && m.is_inter[j] && (m.dirs[i] & 1) && (m.dirs[j] & 2)) {
        m.is_inter[arr] = 1;
        m.dirs[arr] = 3;
        m.f[2 * arr] = m.f[2 * i];
        m.f[2 * arr + 1] = m.f[2 * j + 1];
        const int p0 = E.P.ref_poc[0][m.f[2 * arr].ref], p1 = E.P.ref_poc[1][m.f[2 * arr + 1].ref];
        if (p0 == p1 && m.f[2 * arr].mv[0] == m.f[2 * arr + 1].mv[0] && m.f[2 * arr].mv[1] == m.f[2 * arr + 1].mv[1])
          m.is_inter[arr] = 0;
        else arr++;
      }
    }
  }
  if (arr == maxc) { m.n = arr; return; }
  const int nref = isb ? (E.P.nref[0] < E.P.nref[1] ? E.P.nref[0] : E.P.nref[1]) : E.P.nref[0];
  int r = 0, refcnt = 0;
  while (arr < maxc) {
    m.is_inter[arr] = 1;
    m.dirs[arr] = 1;
    m.f[2 * arr] = MvField{{0, 0}, r};
    if (isb) { m.dirs[arr] = 3; m.f[2 * arr + 1] = MvField{{0, 0}, r}; }
    arr++;
    if (refcnt == nref - 1) r = 0;
    else { r++; refcnt++; }
  }
  m.n = arr;
}

// ============================================================================================
// AMVP: fillMvpCand (TComDataCU.cpp:2623), xAddMVPCand (:2850), xAddMVPCandOrder (:2936)
// ============================================================================================
__device__ int add_mvp(Amvp &in, int list, int ref_idx, const Nb &n) {
  if (!n.valid) return 0;
  const Part &q = n.p[n.idx];
  const int cur_ref_poc = E.P.ref_poc[list][ref_idx];
  if (q.ref[list] >= 0 && cur_ref_poc == E.P.ref_poc[list][q.ref[list]]) {
    in.c[in.n][0] = q.mv[list][0]; in.c[in.n][1] = q.mv[list][1]; in.n++;
    return 1;
  }
  const int l2 = 1 - list;
  if (q.ref[l2] >= 0 && E.P.ref_poc[l2][q.ref[l2]] == cur_ref_poc) {
    in.c[in.n][0] = q.mv[l2][0]; in.c[in.n][1] = q.mv[l2][1]; in.n++;
    return 1;
  }
  return 0;
}
__device__ int add_mvp_order(Amvp &in, int list, int ref_idx, const Nb &n) {
  if (!n.valid) return 0;
  const Part &q = n.p[n.idx];
  const int cur_ref_poc = E.P.ref_poc[list][ref_idx];
  for (int k = 0; k < 2; k++) {
    const int ll = k ? 1 - list : list;
    if (q.ref[ll] >= 0) {
      const int nrp = E.P.ref_poc[ll][q.ref[ll]];
      const int s = dist_scale(E.P.poc, cur_ref_poc, E.P.poc, nrp);
      if (s == 4096) { in.c[in.n][0] = q.mv[ll][0]; in.c[in.n][1] = q.mv[ll][1]; }
      else { in.c[in.n][0] = scale_comp(s, q.mv[ll][0]); in.c[in.n][1] = scale_comp(s, q.mv[ll][1]); }
      in.n++;
      return 1;
    }
  }
  return 0;
}
__device__ void fill_mvp_cand(const Cu *cu, int ps, int pu, int list, int ref_idx, Amvp &in) {
  in.n = 0;
  int lt, rt, lb;
  pu_corners(cu, ps, pu, lt, rt, lb);
  const Nb bl = get_pu_below_left(cu, lb, 1);
  int added_smvp = nb_inter(bl);
  const Nb l = get_pu_left(cu, lb);
  if (!added_smvp) added_smvp = nb_inter(l);
  int added = add_mvp(in, list, ref_idx, bl);
  if (!added) added = add_mvp(in, list, ref_idx, l);
  if (!added) {
    added = add_mvp_order(in, list, ref_idx, bl);
    if (!added) add_mvp_order(in, list, ref_idx, l);
  }
  const Nb ar = get_pu_above_right(cu, rt, 1), a = get_pu_above(cu, rt, 0), al = get_pu_above_left(cu, lt);
  added = add_mvp(in, list, ref_idx, ar);
  if (!added) added = add_mvp(in, list, ref_idx, a);
  if (!added) add_mvp(in, list, ref_idx, al);
  if (!added_smvp) {
    added = add_mvp_order(in, list, ref_idx, ar);
    if (!added) added = add_mvp_order(in, list, ref_idx, a);
    if (!added) add_mvp_order(in, list, ref_idx, al);
  }
  if (in.n == 2 && in.c[0][0] == in.c[1][0] && in.c[0][1] == in.c[1][1]) in.n = 1;
  if (E.P.tmvp) {
    int br_ctu, br_z, c_z;
    col_positions(cu, ps, pu, br_ctu, br_z, c_z);
    int16_t mv[2];
    if ((br_ctu >= 0 && col_mvp(list, br_ctu, br_z, ref_idx, mv)) || col_mvp(list, E.ctu_addr, c_z, ref_idx, mv)) {
      in.c[in.n][0] = mv[0]; in.c[in.n][1] = mv[1]; in.n++;
    }
  }
  if (in.n > 2) in.n = 2;
  while (in.n < 2) { in.c[in.n][0] = in.c[in.n][1] = 0; in.n++; }
}

// ============================================================================================
// Inter residual: encodeResAndCalcRdInterCU (TEncSearch.cpp:4280) with xEstimateInterResidualQT
// (:4426), xEncodeInterResidualQT (:5069), xSetInterResidualQTData (:5157), xAddSymbolBitsInter
// ============================================================================================
template <int LV>
__device__ void encode_inter_residual_qt(const Cu *cu, int comp, const Tu &t) {
  const int rel = tu_abs_rel(t), cur_tr = tu_depth_rel(t);
  const int trmode = cu->p[rel].tr_idx;
  const int subdiv = cur_tr != trmode;
  const int l2 = t.log2;
  if (comp == 3) {
    if (l2 <= 5 && l2 > qt_min_log2(cu, rel)) code_subdiv(subdiv, 5 - l2);
    const int first = cur_tr == 0;
    for (int c = 1; c < 3; c++)
      if (first || t.all[c])
        if (first || cbf_at(&cu->p[rel], c, cur_tr - 1)) code_qt_cbf(cu, t, c, !subdiv);
    if (!subdiv) code_qt_cbf(cu, t, 0, 1);
  }
  if (!subdiv) {
    if (comp != 3 && tu_proc(t, comp))
      if (cbf_at(&cu->p[tu_abs_rel_c(t, comp)], comp, trmode))
        code_coeff_nxn(cu, t, comp, E.S->qt_coef[qt_layer(l2)] + coff(comp) + t.off[comp]);
  } else {
    if (comp == 3 || cbf_at(&cu->p[rel], comp, cur_tr)) {
      if constexpr (LV < 3) {
        TU_LOCAL(ch);
        tu_child(ch, t, 0);
        do encode_inter_residual_qt<LV + 1>(cu, comp, ch); while (tu_next(ch, t));
      } else HMC(false, 22, LV, 0);
    }
  }
}

template <int LV>
__device__ void estimate_inter_residual_qt(Cu *cu, Yuv *resi, double *rd, uint32_t *bits, uint32_t *dist, uint32_t *zero_dist,
                                           const Tu &t) {
  State *S = E.S;
  const int rel = tu_abs_rel(t), depth = tu_depth_total(t), trmode = tu_depth_rel(t), l2 = t.log2;
  const int check_full = l2 <= 5;
  const int check_split = l2 > qt_min_log2(cu, rel);
  double single_cost = kMaxDouble;
  uint32_t single_bits = 0, single_dist = 0;
  uint32_t sdc[3] = {0, 0, 0};
  int32_t abs_sum[3] = {0, 0, 0};
  int best_mode[3] = {0, 0, 0};
  const int layer = qt_layer(l2);
  cload(RD(depth, CI_QT_TRAFO_ROOT), E.cur);
  if (check_full) {
    double min_cost[3] = {kMaxDouble, kMaxDouble, kMaxDouble};
    set_tridx(cu, rel, t.step, trmode);
    reset_bits();
    for (int comp = 0; comp < 3; comp++) {
      if (!tu_proc(t, comp)) continue;
      const int crel = tu_abs_rel_c(t, comp), np = tu_nparts(t, comp);
      const int w = t.w[comp], h = t.h[comp], x0 = t.x0[comp], y0 = t.y0[comp];
      const int check_ts = w <= 4;
      int16_t *cur_coef = S->qt_coef[layer] + coff(comp) + t.off[comp];
      int16_t *qres = yaddr(&S->qt_yuv[layer], comp, x0, y0);
      const int qs = ystride(comp);
      int16_t *pres = yaddr(resi, comp, x0, y0);
      const int modes = check_ts ? 2 : 1;
      int16_t *best_coef = S->rq_best_coef[LV], *best_res = S->rq_best_res[LV];
      for (int mode = 0; mode < modes; mode++) {
        const int first = mode == 0;
        set_ts_range(cu, comp, crel, np, mode);
        cload(E.cur, RD(depth, CI_QT_TRAFO_ROOT));
        reset_bits();
        if (comp != 2) estimate_bit(w, h, comp ? 1 : 0);
        uint32_t cur_bits = 0, cur_dist = 0, non_bits = 0, non_dist = 0;
        double cur_cost = 0, non_cost = 0;
        if (!first) {
          blk_copy(best_coef, w, cur_coef, w, w, h);
          blk_copy(best_res, w, qres, qs, w, h);
        }
        const int32_t cur_abs = transform_tu(cu, t, comp, pres, ystride(comp), cur_coef);
        int32_t cabs = cur_abs;
        if (first || cur_abs == 0) {
          non_dist = weigh(sse_wave(pres, ystride(comp), nullptr, 0, w, h), comp);
          code_qt_cbf_zero(t, comp ? 1 : 0);
          non_bits = written_bits();
          non_cost = rd_cost(non_bits, non_dist);
        }
        if (zero_dist && first) *zero_dist += non_dist;
        if (cur_abs > 0) {
          if (first) {
            cload(E.cur, RD(depth, CI_QT_TRAFO_ROOT));
            reset_bits();
          }
          code_qt_cbf(cu, t, comp, 1);
          code_coeff_nxn(cu, t, comp, cur_coef, true);  // E.td from transform_tu above
          cur_bits = written_bits();
          inv_transform_tu(cu, t, comp, cur_coef, qres, qs, true);
          cur_dist = dist_part(qres, qs, pres, ystride(comp), w, h, comp);
          cur_cost = rd_cost(cur_bits, cur_dist);
        } else if (mode == 1) {
          cur_cost = kMaxDouble;
        } else {
          cur_bits = non_bits; cur_dist = non_dist; cur_cost = non_cost;
        }
        if (cur_cost < min_cost[comp] || (mode == 1 && cur_cost == min_cost[comp])) {
          if (first && (non_cost < cur_cost || cur_abs == 0)) {
            blk_copy(cur_coef, w, nullptr, 0, w, h);
            cabs = 0; cur_bits = non_bits; cur_dist = non_dist; cur_cost = non_cost;
          }
          abs_sum[comp] = cabs;
          sdc[comp] = cur_dist;
          min_cost[comp] = cur_cost;
          best_mode[comp] = mode;
          if (cabs == 0) blk_copy(qres, qs, nullptr, 0, w, h);
        } else {
          blk_copy(cur_coef, w, best_coef, w, w, h);
          blk_copy(qres, qs, best_res, w, w, h);
        }
      }
      set_ts_range(cu, comp, crel, np, best_mode[comp]);
      set_cbf_range(cu, comp, crel, np, (abs_sum[comp] > 0 ? 1 : 0) << trmode);
    }
    cload(E.cur, RD(depth, CI_QT_TRAFO_ROOT));
    reset_bits();
    if (l2 > qt_min_log2(cu, rel)) code_subdiv(0, 5 - l2);
    for (int ch = 0; ch < 3; ch++) {
      const int comp = (ch + 1) == 3 ? 0 : ch + 1;
      if (tu_proc(t, comp)) code_qt_cbf(cu, t, comp, 1);
    }
    for (int comp = 0; comp < 3; comp++)
      if (tu_proc(t, comp)) {
        if (cbf_at(&cu->p[tu_abs_rel_c(t, comp)], comp, trmode))
          code_coeff_nxn(cu, t, comp, S->qt_coef[layer] + coff(comp) + t.off[comp]);
        single_dist += sdc[comp];
      }
    single_bits = written_bits();
    single_cost = rd_cost(single_bits, single_dist);
  }
  if (check_split) {
    if constexpr (LV < 3) {
      if (check_full) {
        cload(RD(depth, CI_QT_TRAFO_TEST), E.cur);
        cload(E.cur, RD(depth, CI_QT_TRAFO_ROOT));
      }
      uint32_t sub_dist = 0, sub_bits = 0;
      double sub_cost = 0;
      int best_cbf[3] = {0, 0, 0};
      for (int c = 0; c < 3; c++)
        if (tu_proc(t, c)) best_cbf[c] = cbf_at(&cu->p[rel], c, trmode);
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      const int qparts = ch.step;
      do estimate_inter_residual_qt<LV + 1>(cu, resi, &sub_cost, &sub_bits, &sub_dist, check_full ? nullptr : zero_dist, ch);
      while (tu_next(ch, t));
      int any = 0;
      for (int c = 0; c < 3; c++) {
        int yuv = 0;
        for (int i = 0; i < 4; i++) yuv |= cbf_at(&cu->p[rel + i * qparts], c, trmode + 1);
        or_cbf_range(cu, c, rel, 4 * qparts, yuv << trmode);
        any |= yuv;
      }
      cload(E.cur, RD(depth, CI_QT_TRAFO_ROOT));
      reset_bits();
      encode_inter_residual_qt<LV>(cu, 3, t);
      for (int c = 0; c < 3; c++) encode_inter_residual_qt<LV>(cu, c, t);
      sub_bits = written_bits();
      sub_cost = rd_cost(sub_bits, sub_dist);
      if (!check_full || (any && sub_cost < single_cost)) {
        *rd += sub_cost; *bits += sub_bits; *dist += sub_dist;
      } else {
        *rd += single_cost; *bits += single_bits; *dist += single_dist;
        set_tridx(cu, rel, t.step, trmode);
        for (int c = 0; c < 3; c++)
          if (tu_proc(t, c)) {
            const int crel = tu_abs_rel_c(t, c), np = tu_nparts(t, c);
            set_cbf_range(cu, c, crel, np, best_cbf[c] << trmode);
            set_ts_range(cu, c, crel, np, best_mode[c]);
          }
        cload(E.cur, RD(depth, CI_QT_TRAFO_TEST));
      }
    } else HMC(false, 23, LV, 0);
  } else {
    *rd += single_cost; *bits += single_bits; *dist += single_dist;
  }
}

template <int LV>
__device__ void set_inter_residual_qt_data(Cu *cu, Yuv *resi, int spatial, const Tu &t) {
  const int rel = tu_abs_rel(t);
  if (tu_depth_rel(t) == cu->p[rel].tr_idx) {
    const int layer = qt_layer(t.log2);
    for (int c = 0; c < 3; c++) {
      if (!tu_proc(t, c)) continue;
      const int w = t.w[c], h = t.h[c];
      if (spatial) blk_copy(yaddr(resi, c, t.x0[c], t.y0[c]), ystride(c), yaddr(&E.S->qt_yuv[layer], c, t.x0[c], t.y0[c]),
                            ystride(c), w, h);
      else blk_copy(cu->coef + coff(c) + t.off[c], w, E.S->qt_coef[layer] + coff(c) + t.off[c], w, w, h);
    }
  } else {
    if constexpr (LV < 3) {
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      do set_inter_residual_qt_data<LV + 1>(cu, resi, spatial, ch); while (tu_next(ch, t));
    } else HMC(false, 24, LV, 0);
  }
}
__device__ void add_symbol_bits_inter(Cu *cu, uint32_t *bits) {
  if (cu->p[0].merge && cu->p[0].part == SIZE_2Nx2N && !cu_qt_root_cbf(cu, 0)) {
    cu_set_all(cu, F_SKIP, 1);
    reset_bits();
    code_skip_flag(cu, 0);
    code_merge_index(cu, 0);
    *bits += written_bits();
  } else {
    reset_bits();
    code_skip_flag(cu, 0);
    code_pred_mode(cu, 0);
    code_part_size(cu, 0, cu->depth);
    encode_pred_info(cu, 0);
    encode_coeff(cu, 0);
    *bits += written_bits();
  }
}
__device__ void clear_residual_fields(Cu *cu) {
  for (int i = lid(); i < cu->nparts; i += 64) {
    Part &p = cu->p[i];
    p.tr_idx = 0;
    p.cbf[0] = p.cbf[1] = p.cbf[2] = 0;
    p.ts[0] = p.ts[1] = p.ts[2] = 0;
  }
  wsync();
}
__device__ __forceinline__ uint8_t *rq_entry(int depth, int k) {
  int off = 0;
  for (int d = 0; d < depth; d++) off += kRqK * rq_entry_bytes(d);
  return E.S->rq_data + off + k * rq_entry_bytes(depth);
}
// the partitions the memo covers (one or two PUs)
__device__ __forceinline__ int rqt_keyed(const Cu *cu) {
  const int ps = cu->p[0].part;
  return ps >= SIZE_2Nx2N && ps <= SIZE_nRx2N && ps != SIZE_NxN;
}
// this lane's word of the memo key: lanes 0-53 the start coder (m_pppcRDSbacCoder[depth]
// [CI_CURR_BEST]), 54-59 the partition and the PUs' motion (a list a PU does not use contributes
// nothing)
__device__ uint32_t rqt_key_word(const Cu *cu) {
  const int l = lid();
  const int ps = cu->p[0].part;
  if (l < 54) return reinterpret_cast<const uint32_t *>(&E.cod[RD(cu->depth, CI_CURR_BEST)])[l];
  const int npu = ps == SIZE_2Nx2N ? 1 : 2;
  uint32_t w[6] = {(uint32_t)ps, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 2; j++) {
    if (j >= npu) break;
    int a, pw, ph;
    part_index_size(cu, ps, j, a, pw, ph);
    const Part &p = cu->p[a];
    const int dir = p.inter_dir;
    w[0] |= (uint32_t)(dir & 3) << (4 + 2 * j);
#pragma unroll
    for (int li = 0; li < 2; li++) {
      const int used = (dir >> li) & 1;
      const uint32_t ref = used ? (uint32_t)(uint8_t)p.ref[li] : 0xffu;
      const int slot = 2 * j + li;  // refs: word 0 bits 8.., the last in word 1
      if (slot < 3) w[0] |= ref << (8 + 8 * slot);
      else w[1] = ref;
      w[2 + slot] = used ? ((uint32_t)(uint16_t)p.mv[li][0] | (uint32_t)(uint16_t)p.mv[li][1] << 16) : 0;
    }
  }
  const int i = l - 54;  // selects, not an indexed (scratch) read
  return i == 0 ? w[0] : i == 1 ? w[1] : i == 2 ? w[2] : i == 3 ? w[3] : i == 4 ? w[4] : i == 5 ? w[5] : 0u;
}
// the entry of this CU whose key equals the lanes' key words, or -1
__device__ __noinline__ int rqt_memo_find(const Cu *cu, int depth) {
  if (!rqt_keyed(cu)) return -1;
  const uint32_t key = rqt_key_word(cu);
  const int n = E.S->rq_n[depth];
  for (int k = 0; k < n; k++) {
    const uint32_t *h = reinterpret_cast<const uint32_t *>(rq_entry(depth, k));
    if (__ballot(lid() < 60 && h[lid()] != key) == 0) return k;
  }
  return -1;
}
__device__ __forceinline__ void cpy64(void *dst, const void *src, int n_int16) {
  uint2 *d = reinterpret_cast<uint2 *>(dst);
  const uint2 *s = reinterpret_cast<const uint2 *>(src);
  for (int i = lid(); i < n_int16 / 4; i += 64) d[i] = s[i];
}
// the residual fields and (unless dropped) coefficients of entry k into the CU
__device__ __noinline__ void rqt_memo_replay(Cu *cu, int depth, int k) {
  const uint8_t *e = rq_entry(depth, k);
  const int np = cu->nparts, W = cu->width, W2 = W * W;
  const uint2 *pp = reinterpret_cast<const uint2 *>(e + 256);
  for (int i = lid(); i < np; i += 64) {
    const uint2 v = pp[i];
    Part &p = cu->p[i];
    p.tr_idx = (int8_t)(v.x & 0xff);
    p.ts[0] = (uint8_t)(v.x >> 8); p.ts[1] = (uint8_t)(v.x >> 16); p.ts[2] = (uint8_t)(v.x >> 24);
    p.cbf[0] = (uint8_t)v.y; p.cbf[1] = (uint8_t)(v.y >> 8); p.cbf[2] = (uint8_t)(v.y >> 16);
  }
  if (!reinterpret_cast<const uint32_t *>(e)[60]) {
    const int16_t *c = reinterpret_cast<const int16_t *>(e + 256 + 8 * np);
    cpy64(cu->coef, c, W2);
    cpy64(cu->coef + coff(1), c + W2, W2 >> 2);
    cpy64(cu->coef + coff(2), c + W2 + (W2 >> 2), W2 >> 2);
  }
  wsync();
}
// a new entry (while the CU has fewer than kRqK): the key, the residual fields, the coefficients
__device__ __noinline__ int rqt_memo_store(const Cu *cu, int depth, int dropped) {
  if (!rqt_keyed(cu)) return -1;
  const int n = E.S->rq_n[depth];
  if (n >= kRqK) return -1;
  const uint32_t key = rqt_key_word(cu);  // recomputed: nothing stays live across the RQT
  uint8_t *e = rq_entry(depth, n);
  const int np = cu->nparts, W = cu->width, W2 = W * W;
  uint32_t *h = reinterpret_cast<uint32_t *>(e);
  if (lid() < 60) h[lid()] = key;
  if (lid() == 60) h[60] = (uint32_t)dropped;
  uint2 *pp = reinterpret_cast<uint2 *>(e + 256);
  for (int i = lid(); i < np; i += 64) {
    const Part &p = cu->p[i];
    pp[i] = make_uint2((uint32_t)(uint8_t)p.tr_idx | (uint32_t)p.ts[0] << 8 | (uint32_t)p.ts[1] << 16 | (uint32_t)p.ts[2] << 24,
                       (uint32_t)p.cbf[0] | (uint32_t)p.cbf[1] << 8 | (uint32_t)p.cbf[2] << 16);
  }
  if (!dropped) {
    int16_t *c = reinterpret_cast<int16_t *>(e + 256 + 8 * np);
    cpy64(c, cu->coef, W2);
    cpy64(c + W2, cu->coef + coff(1), W2 >> 2);
    cpy64(c + W2 + (W2 >> 2), cu->coef + coff(2), W2 >> 2);
  }
  wsync();
  return n;
}
// resi_best of entry k (packed, 1.5 W^2 int16): to = 1 into the entry (and the entry counts from
// now on), 0 out of it
__device__ __noinline__ void rqt_memo_resi(const Cu *cu, int depth, int k, Yuv *resi_best, int to) {
  uint8_t *e = rq_entry(depth, k);
  const int W2 = cu->width * cu->width;
  int16_t *r = reinterpret_cast<int16_t *>(e + 256 + 8 * cu->nparts) + W2 + (W2 >> 1);
  if (to) cpy64(r, resi_best->s, W2 + (W2 >> 1));
  else cpy64(resi_best->s, r, W2 + (W2 >> 1));
  wsync();
}
__device__ void enc_res_rd_inter(Cu *cu, Yuv *org, Yuv *pred, Yuv *resi, Yuv *resi_best, Yuv *reco, int skip_residual) {
  const int W = cu->width, depth = cu->depth;
  if (skip_residual) {
    cu_set_all(cu, F_SKIP, 1);
    yuv_op(YOP_CLEAR, resi, nullptr, nullptr, W);
    yuv_op(YOP_COPY, reco, pred, nullptr, W);
    const uint32_t dist = yuv_dist(reco, org, W);
    E.cur = GOON;
    cload(E.cur, RD(depth, CI_CURR_BEST));
    reset_bits();
    code_skip_flag(cu, 0);
    code_merge_index(cu, 0);
    const uint32_t bits = written_bits();
    const double cost = cu_cost(measure_ssim(cu, org, reco), bits, dist);
    cu->bits = bits; cu->dist = dist; cu->cost = cost;
    cload(RD(depth, CI_TEMP_BEST), E.cur);
    return;
  }
  yuv_op(YOP_SUB, resi, org, pred, W);
  TU_LOCAL(t0);
  tu_root(t0, cu, 0);
  E.cur = GOON;
  cload(E.cur, RD(depth, CI_CURR_BEST));
#define HM_RQT_T0(v) ((void)0)
#define HM_RQT_TADD(c, v) ((void)0)
  HM_RQT_T0(t_find);
  const int hit = rqt_memo_find(cu, depth);
  HM_RQT_TADD(15, t_find);
  int slot = -1;
  if (hit >= 0) {
    HM_RQT_T0(t_rep);
    rqt_memo_replay(cu, depth, hit);
    HM_RQT_TADD(13, t_rep);
  } else
  {
    double nz_cost = 0;
    uint32_t nz_bits = 0, nz_dist = 0, z_dist = 0;
    estimate_inter_residual_qt<0>(cu, resi, &nz_cost, &nz_bits, &nz_dist, &z_dist, t0);
    reset_bits();
    cbin(X_ROOT_CBF, 0);
    const uint32_t zero_bits = written_bits();
    const double zero_cost = rd_cost(zero_bits, z_dist);
    const int dropped = zero_cost < nz_cost || !cu_qt_root_cbf(cu, 0);
    if (dropped) clear_residual_fields(cu);
    else set_inter_residual_qt_data<0>(cu, nullptr, 0, t0);
    HM_RQT_T0(t_st);
    slot = rqt_memo_store(cu, depth, dropped);
    HM_RQT_TADD(14, t_st);
  }
  cload(E.cur, RD(depth, CI_CURR_BEST));
  uint32_t final_bits = 0;
  add_symbol_bits_inter(cu, &final_bits);
  if (!cu_qt_root_cbf(cu, 0)) yuv_op(YOP_CLEAR, resi_best, nullptr, nullptr, W);
  else if (hit >= 0) rqt_memo_resi(cu, depth, hit, resi_best, 0);
  else set_inter_residual_qt_data<0>(cu, resi_best, 1, t0);
  if (slot >= 0) {
    if (cu_qt_root_cbf(cu, 0)) rqt_memo_resi(cu, depth, slot, resi_best, 1);
    if (lid() == 0) E.S->rq_n[depth] = slot + 1;
    wsync();
  }
  cload(RD(depth, CI_TEMP_BEST), E.cur);
  yuv_op(YOP_ADD_CLIP, reco, pred, resi_best, W);
  const uint32_t final_dist = yuv_dist(reco, org, W);
  const double cost = cu_cost(measure_ssim(cu, org, reco), final_bits, final_dist);
  cu->bits = final_bits; cu->dist = final_dist; cu->cost = cost;
}

// ============================================================================================
// predInterSearch (TEncSearch.cpp:2912), P and B slices
// ============================================================================================
__device__ uint32_t template_cost(const Cu *cu, int ps, int pu, Yuv *org, int list, int ref_idx, const int16_t *mvc) {
  HM_PROF(PR_TPL);
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, a, w, h);
  part_position(cu, ps, pu, xp, yp, w, h);
  int mx = mvc[0], my = mvc[1];
  clip_mv(cu, mx, my);
  const int pl = E.P.ref_plane[list][ref_idx];
  int16_t *pr = E.S->mc.pr[0];
  mc_blk(true, E.P.ref16[pl][0], E.P.ref16_stride[0], xp, yp, mx, my, w, h, false, pr, w);
  const int16_t *o = yaddr(org, 0, xp - cu->x, yp - cu->y);
  uint32_t s = 0;
  for (int k = lid(); k < w * h; k += 64) {
    const int r = k / w, c = k - r * w;
    s += (uint32_t)abs((int)pr[k] - (int)o[r * ystride(0) + c]);
  }
  const uint32_t sad = wave_sum_u32(s);
  wsync();
  return (uint32_t)rd_cost_sad(1, sad);
}
// xEstimateMvPredAMVP (:3413); dist_bip (puiDistBiP) takes the best template cost
__device__ void est_mvp_amvp(Cu *cu, int ps, int pu, Yuv *org, int list, int ref_idx, Amvp &in, int16_t *pred, int &mvp_idx,
                             int &mvp_num, uint32_t &dist_bip) {
  fill_mvp_cand(cu, ps, pu, list, ref_idx, in);
  int best = 0;
  if (in.n <= 1) {
    pred[0] = in.c[0][0]; pred[1] = in.c[0][1]; mvp_idx = 0; mvp_num = in.n;
    if (E.P.mvd_l1_zero && list == 1) dist_bip = template_cost(cu, ps, pu, org, list, ref_idx, in.c[0]);
    return;
  }
  uint32_t best_cost = kMaxU32;
  for (int i = 0; i < in.n; i++) {
    const uint32_t c = template_cost(cu, ps, pu, org, list, ref_idx, in.c[i]);
    if (best_cost > c) { best_cost = c; best = i; dist_bip = c; }
  }
  pred[0] = in.c[best][0]; pred[1] = in.c[best][1];
  mvp_idx = best;
  mvp_num = in.n;
}
__device__ void check_best_mvp(const Amvp &in, const int16_t *mv, int16_t *pred, int &mvp_idx, uint32_t &bits, uint32_t &cost) {
  if (in.n < 2) return;
  int best = mvp_idx;
  const int org_bits = (int)(eg_bits(mv[0] - pred[0]) + eg_bits(mv[1] - pred[1])) + 1;
  int best_bits = org_bits;
  for (int i = 0; i < in.n; i++) {
    if (i == mvp_idx) continue;
    const int b = (int)(eg_bits(mv[0] - in.c[i][0]) + eg_bits(mv[1] - in.c[i][1])) + 1;
    if (b < best_bits) { best_bits = b; best = i; }
  }
  if (best != mvp_idx) {
    pred[0] = in.c[best][0]; pred[1] = in.c[best][1];
    mvp_idx = best;
    const uint32_t ob = bits;
    bits = ob - (uint32_t)org_bits + (uint32_t)best_bits;
    cost = (cost - mv_cost_bits(ob)) + mv_cost_bits(bits);
  }
}
// xMotionEstimation (uni): TZ search + fractional refinement through hvx_me.hpp
__device__ void motion_estimation(Cu *cu, int ps, int pu, int list, int ref_idx, const int16_t *pred, int16_t *mv,
                                  uint32_t &bits, uint32_t &cost) {
  HM_PROF(PR_ME);
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, a, w, h);
  part_position(cu, ps, pu, xp, yp, w, h);
  hvx_me_job j;
  memset(&j, 0, sizeof(j));
  j.pic_w = E.P.w; j.pic_h = E.P.h; j.max_cu = 64;
  j.cu_x = cu->x; j.cu_y = cu->y;
  j.pu_x = xp; j.pu_y = yp; j.w = w; j.h = h;
  j.pred_x = pred[0]; j.pred_y = pred[1];
  j.use_int2nx2n = (ps != SIZE_2Nx2N || cu->depth != 0);
  j.i2_x = E.S->int2n[list][ref_idx][0];
  j.i2_y = E.S->int2n[list][ref_idx][1];
  j.bits_in = (int32_t)bits;
  j.search_range = E.P.search_range;
  j.lambda_motion = E.P.lambda_motion;
  j.flags = HVX_ME_FEN | HVX_ME_HADME | HVX_ME_SMOOTHMV;
  const int pi = E.P.ref_plane[list][ref_idx];
  HMC(pi >= 0 && pi < 8 && E.P.ref8[pi] != nullptr && xp >= 0 && yp >= 0 && xp + w <= E.P.w && yp + h <= E.P.h, 6, pi,
      xp * 10000 + yp);
  MeScratch &ms = E.S->me;
  const uint8_t *org = E.P.org[0] + yp * E.P.org_stride[0] + xp;
  const int os = E.P.org_stride[0];
  for (int k = lid(); k < w * h; k += 64) {
    const int y = k / w, x = k - y * w;
    ms.sm.org[y * 64 + x] = org[y * os + x];
  }
  wsync();
  MeInt m;
  m.org = ms.sm.org; m.red = ms.red; m.par = 0; m.os = 64;
  me_ref_setup(m, j, E.P.ref8[pi], E.P.ref8_stride);
  const bool spec = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
  m.sub = (h > 8 && spec) ? 1 : 0;
  m.rows = (h + (1 << m.sub) - 1) >> m.sub;
  m.gw = w >> 2;
  m.lam = j.lambda_motion;
  m.px = j.pred_x; m.py = j.pred_y;
  me_tz<0, 0, 1>(j, m);
  const uint32_t sad_int = m.best_sad - me_mv_cost(m.lam, m.px, m.py, 2, m.best_x, m.best_y);
  me_frac_refine<64, 1, true, uint8_t>(j, m.ref, E.P.ref8_stride, m.best_x, m.best_y, sad_int, ms.sm, &ms.r);
  wsync();
  const hvx_me_result r = ms.r;
  wsync();
  // the block the result points at lies inside the reference plane's margin (HVX_PLANE_MARGIN 80)
  HMC(4 * xp + r.mv_x >= -4 * 80 && 4 * yp + r.mv_y >= -4 * 80 && 4 * (xp + w) + r.mv_x <= 4 * (E.P.w + 80) &&
          4 * (yp + h) + r.mv_y <= 4 * (E.P.h + 80),
      9, r.mv_x, r.mv_y);
  if (ps == SIZE_2Nx2N) { E.S->int2n[list][ref_idx][0] = (int16_t)r.mv_int_x; E.S->int2n[list][ref_idx][1] = (int16_t)r.mv_int_y; }
  mv[0] = (int16_t)r.mv_x; mv[1] = (int16_t)r.mv_y;
  bits = r.bits;
  cost = r.cost;
}
// xMergeEstimation (:2832)
__device__ void merge_estimation(Cu *cu, int ps, int pu, Yuv *org, int &inter_dir, MvField *mf, int &merge_idx, uint32_t &cost,
                                 MergeList &m) {
  int a, w, h;
  part_index_size(cu, ps, pu, a, w, h);
  merge_candidates(cu, ps, pu, m);
  const int n = m.n;
  if (cu->width == 8 && (w < 8 || h < 8))
    for (int i = 0; i < n; i++)
      if (m.dirs[i] == 3) { m.dirs[i] = 1; m.f[2 * i + 1] = MvField{{0, 0}, -1}; }
  cost = kMaxU32;
  int xp, yp;
  part_position(cu, ps, pu, xp, yp, w, h);
  for (int i = 0; i < n; i++) {
    pu_set_mvfield(cu, ps, pu, 0, m.f[2 * i].mv[0], m.f[2 * i].mv[1], m.f[2 * i].ref);
    pu_set_mvfield(cu, ps, pu, 1, m.f[2 * i + 1].mv[0], m.f[2 * i + 1].mv[1], m.f[2 * i + 1].ref);
    mc_pu(cu, ps, pu, &E.S->tmp_yuv_pred);
    uint32_t c = wave_satd(yaddr(org, 0, xp - cu->x, yp - cu->y), ystride(0), yaddr(&E.S->tmp_yuv_pred, 0, xp - cu->x, yp - cu->y),
                           ystride(0), w, h);
    uint32_t b = (uint32_t)i + 1;
    if (i == E.P.max_merge - 1) b--;
    c += mv_cost_bits(b);
    if (c < cost) {
      cost = c;
      mf[0] = m.f[2 * i];
      mf[1] = m.f[2 * i + 1];
      inter_dir = m.dirs[i];
      merge_idx = i;
    }
  }
}
// xMotionEstimation with bBi (TEncSearch.cpp:3686-3696, :3710-3712, :3726-3729, :3759): the target
// is 2 * org - m_acYuvPred[other list] (TComYuv::removeHighFreq, TComYuv.cpp:409; unclipped:
// ClipForBiPredMEEnabled is off), xPatternSearch over +-BipredSearchRange around the list's current
// MV (rcMv on entry), the fractional refinement on the same int16 target, the cost weighted by 0.5.
// One candidate point per lane (raster order, first minimum as in k_me_full).
__device__ void motion_estimation_bi(Cu *cu, int ps, int pu, Yuv *org, int list, int ref_idx, const int16_t *pred,
                                     int16_t *mv, uint32_t &bits, uint32_t &cost) {
  HM_PROF(PR_ME);
  int a, w, h, xp, yp;
  part_index_size(cu, ps, pu, a, w, h);
  part_position(cu, ps, pu, xp, yp, w, h);
  const int rx = xp - cu->x, ry = yp - cu->y;
  MeFracSmem<64, 1, int16_t> &sm = E.S->me.sm16;
  const int16_t *o = yaddr(org, 0, rx, ry), *q = E.S->pred_l[1 - list] + ry * 64 + rx;
  for (int k = lid(); k < w * h; k += 64) {
    const int y = k / w, x = k - y * w;
    sm.org[y * 64 + x] = (int16_t)(2 * o[y * ystride(0) + x] - q[y * 64 + x]);
  }
  wsync();
  hvx_me_job j;
  memset(&j, 0, sizeof(j));
  j.pic_w = E.P.w; j.pic_h = E.P.h; j.max_cu = 64;
  j.cu_x = cu->x; j.cu_y = cu->y;
  j.pu_x = xp; j.pu_y = yp; j.w = w; j.h = h;
  j.pred_x = pred[0]; j.pred_y = pred[1];
  j.center_x = mv[0]; j.center_y = mv[1];
  j.bits_in = (int32_t)bits;
  j.search_range = E.P.bipred_range;
  j.lambda_motion = E.P.lambda_motion;
  j.flags = HVX_ME_FEN | HVX_ME_HADME | HVX_ME_BI;
  const int pi = E.P.ref_plane[list][ref_idx];
  const int stride = E.P.ref8_stride;
  const uint8_t *ref = E.P.ref8[pi] + yp * stride + xp;
  const MeRange g = me_search_range(j, j.center_x, j.center_y, j.search_range);
  // FEN subsamples rows when iRows > 8 (:3810); only the specialised SAD widths honour it
  const bool spec = (w == 4 || w == 8 || w == 16 || w == 32 || w == 64 || w == 12 || w == 24 || w == 48);
  const int sub = (h > 8 && spec) ? 1 : 0;
  const int nx = g.r - g.l + 1, np = nx * (g.b - g.t + 1);
  uint64_t best = ~0ull;
  for (int p = lid(); p < np; p += 64) {
    const int py = p / nx, x = g.l + (p - py * nx), y = g.t + py;
    const uint8_t *r = ref + y * stride + x;
    uint32_t sad = 0;
    for (int row = 0; row < h; row += 1 << sub)
      for (int c = 0; c < w; c++) sad += (uint32_t)abs((int)sm.org[row * 64 + c] - (int)r[row * stride + c]);
    const uint32_t c = (sad << sub) + me_mv_cost(j.lambda_motion, j.pred_x, j.pred_y, 2, x, y);
    const uint64_t key = ((uint64_t)c << 32) | (uint32_t)p;
    best = key < best ? key : best;
  }
  best = wave_min_u64(best);
  const int bp = (int)(uint32_t)best, by = bp / nx;
  const int ix = g.l + (bp - by * nx), iy = g.t + by;
  const uint32_t sad_int = (uint32_t)(best >> 32) - me_mv_cost(j.lambda_motion, j.pred_x, j.pred_y, 2, ix, iy);
  me_frac_refine<64, 1, true, int16_t>(j, ref, stride, ix, iy, sad_int, sm, &E.S->me.r);
  wsync();
  const hvx_me_result r = E.S->me.r;
  wsync();
  // the block the vector points at stays inside the padded reference (as check 9: clipMv allows
  // up to -(x + 72) samples, so the vector itself is not bounded by the margin)
  HMC(4 * xp + r.mv_x >= -4 * 80 && 4 * yp + r.mv_y >= -4 * 80 && 4 * (xp + w) + r.mv_x <= 4 * (E.P.w + 80) &&
          4 * (yp + h) + r.mv_y <= 4 * (E.P.h + 80), 10, r.mv_x, r.mv_y);
  mv[0] = (int16_t)r.mv_x; mv[1] = (int16_t)r.mv_y;
  bits = r.bits;
  cost = r.cost;
}
// xGetBlkBits (:3509)
__device__ __forceinline__ void blk_bits(int ps, int is_p, int pu, int last_mode, uint32_t *b) {
  if (ps == SIZE_2Nx2N || ps == SIZE_NxN) { b[0] = is_p ? 1 : 3; b[1] = 3; b[2] = 5; return; }
  if (is_p) { b[0] = 3; b[1] = 0; b[2] = 0; return; }
  const bool hor = ps == SIZE_2NxN || ps == SIZE_2NxnU || ps == SIZE_2NxnD;
  if (pu == 0) { b[0] = 0; b[1] = (hor || last_mode != 0) ? 0 : 2; b[2] = last_mode == 0 ? 3 : 0; return; }
  // PU 1: {5,7,7} after uni-L0, {7,5,7} (2NxN) / {5,5,7} (Nx2N) after uni-L1, {6,6,6} after bi
  if (last_mode == 2) { b[0] = b[1] = b[2] = 6; return; }
  b[0] = (last_mode == 1 && hor) ? 7 : 5;
  b[1] = last_mode == 0 ? 7 : 5;
  b[2] = 7;
}
// the reference index bits of predInterSearch (:3021-3028)
__device__ __forceinline__ uint32_t ref_bits(int r, int n) { return n <= 1 ? 0u : (uint32_t)r + 1 - (r == n - 1 ? 1u : 0u); }
__device__ void pred_inter_search(Cu *cu, Yuv *org, Yuv *pred, int use_mrg) {
  const int ps = cu->p[0].part, npart = num_parts_of(ps);
  const int isb = E.P.slice_type == B_SLICE, ndir = isb ? 2 : 1;
  InterSearch &Q = E.is;
  int last_mode = 0;
  // declared before the PU loop in the reference (:2937-2969): carried across the PUs
  int best_bip_ref_l1 = 0, best_bip_mvp_l1 = 0;
  uint32_t bip_dist_temp = kMaxU32;
  Q.mv[0][0] = Q.mv[0][1] = Q.mv[1][0] = Q.mv[1][1] = 0;
  Q.ref[0] = Q.ref[1] = 0;
  for (int pu = 0; pu < npart; pu++) {
    Q.cost[0] = Q.cost[1] = kMaxU32;
    Q.bits[0] = Q.bits[1] = Q.bits[2] = 0;
    uint32_t cost_bi = kMaxU32, best_bip_dist = kMaxU32;
    for (int r = 0; r < 4; r++) { Q.cost_l0[r] = kMaxU32; Q.bits_l0[r] = 0; }
    int16_t mv_valid_l1[2] = {0, 0};
    int ref_valid_l1 = 0;
    uint32_t bits_valid_l1 = kMaxU32, cost_valid_l1 = kMaxU32;
    Q.mvbi[0][0] = Q.mvbi[0][1] = Q.mvbi[1][0] = Q.mvbi[1][1] = 0;
    Q.refbi[0] = Q.refbi[1] = 0;
    uint32_t mb[3];
    blk_bits(ps, !isb, pu, last_mode, mb);
    int a, w, h;
    part_index_size(cu, ps, pu, a, w, h);
    const int test_normal = !(use_mrg && cu->width > 8 && npart == 2);
    if (test_normal) {
      // uni-directional prediction (:3014-3093)
      for (int l = 0; l < ndir; l++) {
        const int nref = E.P.nref[l];
        for (int r = 0; r < nref; r++) {
          uint32_t bt = mb[l] + ref_bits(r, nref), ct;
          int pidx, pnum;
          est_mvp_amvp(cu, ps, pu, org, l, r, Q.amvp[l][r], Q.mvpred[l][r], pidx, pnum, bip_dist_temp);
          pu_set(cu, ps, pu, PU_MVP_IDX, l, pidx);
          pu_set(cu, ps, pu, PU_MVP_NUM, l, pnum);
          if (E.P.mvd_l1_zero && l == 1 && bip_dist_temp < best_bip_dist) {
            best_bip_dist = bip_dist_temp;
            best_bip_mvp_l1 = pidx;
            best_bip_ref_l1 = r;
          }
          bt += 1;  // m_auiMVPIdxCost[idx][AMVP_MAX_NUM_CANDS]
          const int m = l == 1 ? E.P.l1_to_l0[r] : -1;
          if (m >= 0) {
            // FastMEForGenBLowDelayEnabled (:3042-3055): list 0's search of the same picture, re-costed
            Q.mvtemp[1][r][0] = Q.mvtemp[0][m][0]; Q.mvtemp[1][r][1] = Q.mvtemp[0][m][1];
            ct = Q.cost_l0[m] - mv_cost_bits(Q.bits_l0[m]);
            bt += eg_bits(Q.mvtemp[1][r][0] - Q.mvpred[1][r][0]) + eg_bits(Q.mvtemp[1][r][1] - Q.mvpred[1][r][1]);
            ct += mv_cost_bits(bt);
          } else {
            motion_estimation(cu, ps, pu, l, r, Q.mvpred[l][r], Q.mvtemp[l][r], bt, ct);
          }
          check_best_mvp(Q.amvp[l][r], Q.mvtemp[l][r], Q.mvpred[l][r], pidx, bt, ct);
          Q.mvp_idx[l][r] = pidx; Q.mvp_num[l][r] = pnum;
          if (l == 0) { Q.cost_l0[r] = ct; Q.bits_l0[r] = bt; }
          if (ct < Q.cost[l]) {
            Q.cost[l] = ct; Q.bits[l] = bt;
            Q.mv[l][0] = Q.mvtemp[l][r][0]; Q.mv[l][1] = Q.mvtemp[l][r][1];
            Q.ref[l] = r;
          }
          if (l == 1 && ct < cost_valid_l1 && m < 0) {
            cost_valid_l1 = ct; bits_valid_l1 = bt;
            mv_valid_l1[0] = Q.mvtemp[l][r][0]; mv_valid_l1[1] = Q.mvtemp[l][r][1];
            ref_valid_l1 = r;
          }
        }
      }
      // bi-directional prediction (:3096-3251); UseFastEnc: one iteration
      if (isb && !(cu->width == 8 && (w < 8 || h < 8))) {  // isBipredRestriction (TComDataCU.cpp:2773)
        for (int l = 0; l < 2; l++) {
          Q.mvbi[l][0] = Q.mv[l][0]; Q.mvbi[l][1] = Q.mv[l][1];
          Q.refbi[l] = Q.ref[l];
          for (int r = 0; r < 4; r++) {
            Q.mvpredbi[l][r][0] = Q.mvpred[l][r][0]; Q.mvpredbi[l][r][1] = Q.mvpred[l][r][1];
            Q.mvp_idx_bi[l][r] = Q.mvp_idx[l][r];
          }
        }
        if (E.P.mvd_l1_zero) {
          const int br = best_bip_ref_l1;
          pu_set(cu, ps, pu, PU_MVP_IDX, 1, best_bip_mvp_l1);
          Q.mvp_idx_bi[1][br] = best_bip_mvp_l1;
          Q.mvpredbi[1][br][0] = Q.amvp[1][br].c[best_bip_mvp_l1][0];
          Q.mvpredbi[1][br][1] = Q.amvp[1][br].c[best_bip_mvp_l1][1];
          Q.mvbi[1][0] = Q.mvpredbi[1][br][0]; Q.mvbi[1][1] = Q.mvpredbi[1][br][1];
          Q.refbi[1] = br;
          pu_set_mvfield(cu, ps, pu, 1, Q.mvbi[1][0], Q.mvbi[1][1], br);
          mc_pu_list_luma(cu, ps, pu, 1, E.S->pred_l[1]);
          Q.motbits[0] = Q.bits[0] - mb[0];
          Q.motbits[1] = mb[1] + ref_bits(br, E.P.nref[1]) + 1;
          Q.bits[2] = mb[2] + Q.motbits[0] + Q.motbits[1];
          Q.mvtemp[1][br][0] = Q.mvbi[1][0]; Q.mvtemp[1][br][1] = Q.mvbi[1][1];
        } else {
          Q.motbits[0] = Q.bits[0] - mb[0];
          Q.motbits[1] = Q.bits[1] - mb[1];
          Q.bits[2] = mb[2] + Q.motbits[0] + Q.motbits[1];
        }
        int l = Q.cost[0] <= Q.cost[1] ? 1 : 0;
        if (!E.P.mvd_l1_zero) {
          pu_set_mv(cu, ps, pu, 1 - l, Q.mv[1 - l][0], Q.mv[1 - l][1]);
          pu_set_ref(cu, ps, pu, 1 - l, Q.ref[1 - l]);
          mc_pu_list_luma(cu, ps, pu, 1 - l, E.S->pred_l[1 - l]);
        } else l = 0;
        int changed = 0;
        const int nref = E.P.nref[l];
        for (int r = 0; r < nref; r++) {
          uint32_t bt = mb[2] + Q.motbits[1 - l] + ref_bits(r, nref) + 1, ct;
          motion_estimation_bi(cu, ps, pu, org, l, r, Q.mvpredbi[l][r], Q.mvtemp[l][r], bt, ct);
          int pidx = Q.mvp_idx_bi[l][r];
          check_best_mvp(Q.amvp[l][r], Q.mvtemp[l][r], Q.mvpredbi[l][r], pidx, bt, ct);
          Q.mvp_idx_bi[l][r] = pidx;
          if (ct < cost_bi) {
            changed = 1;
            Q.mvbi[l][0] = Q.mvtemp[l][r][0]; Q.mvbi[l][1] = Q.mvtemp[l][r][1];
            Q.refbi[l] = r;
            cost_bi = ct;
            Q.motbits[l] = bt - mb[2] - Q.motbits[1 - l];
            Q.bits[2] = bt;
          }
        }
        if (!changed && cost_bi <= Q.cost[0] && cost_bi <= Q.cost[1]) {
          for (int k = 0; k < (E.P.mvd_l1_zero ? 1 : 2); k++) {
            int pidx = Q.mvp_idx_bi[k][Q.refbi[k]];
            uint32_t b2 = Q.bits[2];
            check_best_mvp(Q.amvp[k][Q.refbi[k]], Q.mvbi[k], Q.mvpredbi[k][Q.refbi[k]], pidx, b2, cost_bi);
            Q.bits[2] = b2;
            Q.mvp_idx_bi[k][Q.refbi[k]] = pidx;
          }
        }
      }
    }
    // clear the PU's motion (:3257-3265)
    pu_set_mvfield(cu, ps, pu, 0, 0, 0, -1);
    pu_set_mvfield(cu, ps, pu, 1, 0, 0, -1);
    pu_set_mvd(cu, ps, pu, 0, 0, 0);
    pu_set_mvd(cu, ps, pu, 1, 0, 0);
    pu_set(cu, ps, pu, PU_MVP_IDX, 0, -1); pu_set(cu, ps, pu, PU_MVP_NUM, 0, -1);
    pu_set(cu, ps, pu, PU_MVP_IDX, 1, -1); pu_set(cu, ps, pu, PU_MVP_NUM, 1, -1);
    uint32_t me_bits = 0;
    // list 1 alone only through a picture list 0 does not hold (:3269-3272)
    Q.mv[1][0] = mv_valid_l1[0]; Q.mv[1][1] = mv_valid_l1[1];
    Q.ref[1] = ref_valid_l1;
    Q.bits[1] = bits_valid_l1;
    Q.cost[1] = cost_valid_l1;
    if (test_normal) {
      if (cost_bi <= Q.cost[0] && cost_bi <= Q.cost[1]) {
        last_mode = 2;
        const int r0 = Q.refbi[0], r1 = Q.refbi[1];
        pu_set_mv(cu, ps, pu, 0, Q.mvbi[0][0], Q.mvbi[0][1]);
        pu_set_ref(cu, ps, pu, 0, r0);
        pu_set_mv(cu, ps, pu, 1, Q.mvbi[1][0], Q.mvbi[1][1]);
        pu_set_ref(cu, ps, pu, 1, r1);
        pu_set_mvd(cu, ps, pu, 0, Q.mvbi[0][0] - Q.mvpredbi[0][r0][0], Q.mvbi[0][1] - Q.mvpredbi[0][r0][1]);
        pu_set_mvd(cu, ps, pu, 1, Q.mvbi[1][0] - Q.mvpredbi[1][r1][0], Q.mvbi[1][1] - Q.mvpredbi[1][r1][1]);
        pu_set(cu, ps, pu, PU_INTER_DIR, 0, 3);
        pu_set(cu, ps, pu, PU_MVP_IDX, 0, Q.mvp_idx_bi[0][r0]);
        pu_set(cu, ps, pu, PU_MVP_NUM, 0, Q.mvp_num[0][r0]);
        pu_set(cu, ps, pu, PU_MVP_IDX, 1, Q.mvp_idx_bi[1][r1]);
        pu_set(cu, ps, pu, PU_MVP_NUM, 1, Q.mvp_num[1][r1]);
        me_bits = Q.bits[2];
      } else {
        const int l = Q.cost[0] <= Q.cost[1] ? 0 : 1;
        last_mode = l;
        const int r = Q.ref[l];
        pu_set_mv(cu, ps, pu, l, Q.mv[l][0], Q.mv[l][1]);
        pu_set_ref(cu, ps, pu, l, r);
        pu_set_mvd(cu, ps, pu, l, Q.mv[l][0] - Q.mvpred[l][r][0], Q.mv[l][1] - Q.mvpred[l][r][1]);
        pu_set(cu, ps, pu, PU_INTER_DIR, 0, l + 1);
        pu_set(cu, ps, pu, PU_MVP_IDX, l, Q.mvp_idx[l][r]);
        pu_set(cu, ps, pu, PU_MVP_NUM, l, Q.mvp_num[l][r]);
        me_bits = Q.bits[l];
      }
    }
    if (ps != SIZE_2Nx2N) {
      uint32_t me_cost = kMaxU32;
      int xp, yp;
      part_position(cu, ps, pu, xp, yp, w, h);
      if (test_normal) {
        mc_pu(cu, ps, pu, &E.S->tmp_yuv_pred);
        const uint32_t err = wave_satd(yaddr(org, 0, xp - cu->x, yp - cu->y), ystride(0),
                                       yaddr(&E.S->tmp_yuv_pred, 0, xp - cu->x, yp - cu->y), ystride(0), w, h);
        me_cost = err + mv_cost_bits(me_bits);
      }
      const Part save = cu->p[a];
      int mrg_dir = 0, mrg_idx = 0;
      MvField mrg[2] = {MvField{{0, 0}, -1}, MvField{{0, 0}, -1}};
      uint32_t mrg_cost = kMaxU32;
      MergeList ml;
      merge_estimation(cu, ps, pu, org, mrg_dir, mrg, mrg_idx, mrg_cost, ml);
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
    mc_pu(cu, ps, pu, pred);
  }
}

// ============================================================================================
// Intra: reference samples, prediction, xIntraCodingTUBlock and the luma / chroma RD searches
// ============================================================================================
// the availability flags of a TU's neighbour units (TComPattern.cpp:570-760), one lane per unit
__device__ void intra_avail(const Cu *cu, const Tu &t, int comp) {
  const int w = t.w[comp], h = t.h[comp];
  const int unit = comp ? 2 : 4;
  const int wu = w / unit, hu = h / unit;
  const int lt = cu->zidx + tu_abs_rel(t);
  const int rlt = z2r(lt);
  const int rt = r2z(rlt + wu - 1), lb = r2z(rlt + (hu - 1) * 16);
  const int lunits = hu * 2, total = lunits + 1 + 2 * wu;
  const int k = lid();
  int v = 0;
  if (k < total) {
    if (k < hu) v = get_pu_below_left(cu, lb, hu - k).valid;
    else if (k < lunits) v = get_pu_left(cu, r2z(rlt + (lunits - 1 - k) * 16)).valid;
    else if (k == lunits) v = get_pu_above_left(cu, lt).valid;
    else if (k <= lunits + wu) v = get_pu_above(cu, r2z(rlt + (k - lunits - 1)), 0).valid;
    else v = get_pu_above_right(cu, rt, k - lunits - wu).valid;
  }
  const uint64_t m = __ballot(v);
  wsync();
  E.avail[0] = (uint32_t)m;
  E.avail[1] = (uint32_t)(m >> 32);
  E.avail[2] = 0;
  wsync();
}
// fillReferenceSamples (TComPattern.cpp:364) of the TU into B (unfiltered), from the reconstruction
__device__ void intra_border(const Cu *cu, const Tu &t, int comp, int16_t *B) {
  intra_avail(cu, t, comp);
  const int c = comp, s = c ? 1 : 0, n = t.w[c], ulog2 = c ? 1 : 2, u = 1 << ulog2;
  const int x0 = (cu->x >> s) + t.x0[c], y0 = (cu->y >> s) + t.y0[c];
  const int nunits = ((4 * n) >> ulog2) + 1;
  uint32_t a[3];
  int navail = 0;
  for (int w = 0; w < 3; w++) {
    const int lo = w * 32;
    a[w] = nunits >= lo + 32 ? E.avail[w] : nunits > lo ? E.avail[w] & ((1u << (nunits - lo)) - 1u) : 0u;
    navail += __popc(a[w]);
  }
  auto line = [&](int l) {  // HM's reference line: bottom-left upwards, above-left unit, above row
    if (l < 2 * n) return rec_px(c, x0 - 1, y0 + 2 * n - 1 - l);
    if (l < 2 * n + u) return rec_px(c, x0 - 1, y0 - 1);
    return rec_px(c, x0 + (l - 2 * n - u), y0 - 1);
  };
  for (int k = lid(); k <= 4 * n; k += 64) {
    const int l = k == 0 ? 2 * n + u - 1 : k <= 2 * n ? 2 * n + u + k - 1 : 4 * n - k;
    int v = 128;
    if (navail) {
      const int uu = l >> ulog2;
      if ((a[uu >> 5] >> (uu & 31)) & 1) v = line(l);
      else {
        const int j = intra::highest_below(a, uu);
        v = j >= 0 ? line(j * u + u - 1) : line(intra::lowest_above(a, uu) * u);
      }
    }
    B[k] = (int16_t)v;
  }
  wsync();
}
// predIntraAng of a TU into pred (stride ystride(comp))
__device__ void intra_predict_tu(const Cu *cu, const Tu &t, int comp, int mode, int16_t *pred) {
  HM_PROF(PR_IPRED);
  IntraScratch &is = E.u.in;
  uint8_t *is_org = is.org;
  const int n = t.w[comp], log2n = ilog2(n);
  const bool luma = comp == 0;
  intra_border(cu, t, comp, is.unf);
  const bool filt = luma && intra::use_filter(mode, log2n, true);
  if (filt) {
    intra::filter_border(is.unf, n, log2n, true, true, is.filt);
    wsync();
  }
  const int dc = intra::dc_value(is.unf, n, log2n);
  const intra::Mode md(mode);
  const int16_t *B = filt ? is.filt : is.unf;
  const bool edge = luma && n <= 16;
  const int ps = ystride(comp);
  for (int k = lid(); k < n * n; k += 64) {
    const int r = k >> log2n, cc = k & (n - 1);
    pred[r * ps + cc] = (int16_t)intra::pred_sample(B, n, log2n, md, edge, dc, r, cc);
  }
  wsync();
}

// the first pass of estIntraPredLumaQT (:2221-2330): SATD of 35 modes + xModeBitsIntra, the
// candidate list and the MPM append (HHI_RQT_INTRA_SPEEDUP, FastUDIUseMPM)
__device__ void intra_first_pass(const Cu *cu, const Tu &tpu, Yuv *org, int depth) {
  HM_PROF(PR_IFP);
  IntraScratch &is = E.u.in;
  uint8_t *is_org = is.org;
  const int n = tpu.w[0], log2n = ilog2(n);
  intra_border(cu, tpu, 0, is.unf);
  intra::filter_border(is.unf, n, log2n, true, true, is.filt);
  for (int k = lid(); k < n * n; k += 64) is_org[k] = (uint8_t)*yaddr(org, 0, tpu.x0[0] + (k & (n - 1)), tpu.y0[0] + (k >> log2n));
  if (lid() < 36) is.satd[lid()] = 0;
  wsync();
  const int dc = intra::dc_value(is.unf, n, log2n);
  const bool edge = n <= 16;
  const int lt = n == 4 ? 2 : 3, tt = 1 << lt, tps = n >> lt, ntile = tps * tps;
  for (int idx = lid(); idx < 35 * ntile; idx += 64) {
    const int m = idx / ntile, ti = idx - m * ntile, r0 = (ti / tps) << lt, c0 = (ti % tps) << lt;
    const intra::Mode md(m);
    const int16_t *B = intra::use_filter(m, log2n, true) ? is.filt : is.unf;
    uint32_t sum = 0;
    if (tt == 8) {
      int d[8][8];
      for (int y = 0; y < 8; y++) {
        int row[8];
        for (int x = 0; x < 8; x++)
          row[x] = (int)is_org[(r0 + y) * n + c0 + x] - intra::pred_sample(B, n, log2n, md, edge, dc, r0 + y, c0 + x);
        hadamard8(row, d[y]);
      }
      for (int x = 0; x < 8; x++) {
        int col[8], rr[8];
        for (int y = 0; y < 8; y++) col[y] = d[y][x];
        hadamard8(col, rr);
        for (int k = 0; k < 8; k++) sum += (uint32_t)abs(rr[k]);
      }
      sum = (sum + 2) >> 2;
    } else {
      int d[4][4];
      for (int y = 0; y < 4; y++) {
        int row[4];
        for (int x = 0; x < 4; x++) row[x] = (int)is_org[y * 4 + x] - intra::pred_sample(B, 4, 2, md, edge, dc, y, x);
        hadamard4(row, d[y]);
      }
      for (int x = 0; x < 4; x++) {
        int col[4] = {d[0][x], d[1][x], d[2][x], d[3][x]}, rr[4];
        hadamard4(col, rr);
        for (int k = 0; k < 4; k++) sum += (uint32_t)abs(rr[k]);
      }
      sum = (sum + 1) >> 1;
    }
    atomicAdd(&is.satd[m], sum);
  }
  wsync();
  // rates, costs, ranking, MPM append (every lane the same scalar steps)
  const int poff = tu_abs_rel(tpu);
  const Nb l = get_pu_left(cu, cu->zidx + poff), a = get_pu_above(cu, cu->zidx + poff, 1);
  const int ld = (l.valid && l.p[l.idx].pred == MODE_INTRA) ? l.p[l.idx].idir[0] : 1;
  const int ad = (a.valid && a.p[a.idx].pred == MODE_INTRA) ? a.p[a.idx].idir[0] : 1;
  int imode, mp0, mp1, mp2;
  if (ld == ad) {
    imode = 1;
    if (ld > 1) { mp0 = ld; mp1 = ((ld + 29) % 32) + 2; mp2 = ((ld - 1) % 32) + 2; }
    else { mp0 = 0; mp1 = 1; mp2 = 26; }
  } else {
    imode = 2;
    mp0 = ld; mp1 = ad;
    mp2 = (ld && ad) ? 0 : ((ld + ad) < 2 ? 26 : 1);
  }
  int num = intra::kNumRdMpm[log2n - 1];
  int *list = is.list;
  double *cc = is.cc;
  wsync();
  for (int k = 0; k < 10; k++) { list[k] = 0; cc[k] = 1.7976931348623157e308; }
  list[10] = list[11] = 0;
  const Coder &cb = E.cod[RD(depth, CI_CURR_BEST)];
  const uint64_t frac = (uint64_t)(uint32_t)(cb.frac & 32767);
  const int st = cb.st[X_INTRA] & 127;
  const uint64_t eb_mpm = (uint64_t)ebits(st ^ 1), eb_no = (uint64_t)ebits(st);
  for (int m = 0; m < 35; m++) {
    const int idx = m == mp0 ? 0 : m == mp1 ? 1 : m == mp2 ? 2 : -1;
    const uint64_t total = frac + (idx >= 0 ? eb_mpm : eb_no) + 32768ull * (uint64_t)(idx < 0 ? 5 : idx ? 2 : 1);
    const uint32_t bits = (uint32_t)(total >> 15);
    const double cost = __dadd_rn((double)is.satd[m], __dmul_rn((double)bits, E.P.sqrt_lambda));
    int sh = 0;
    while (sh < num && cost < cc[num - 1 - sh]) sh++;
    if (sh) {
      for (int k = 1; k < sh; k++) { list[num - k] = list[num - 1 - k]; cc[num - k] = cc[num - 1 - k]; }
      list[num - sh] = m;
      cc[num - sh] = cost;
    }
  }
  for (int q = 0; q < imode; q++) {
    const int mq = q == 0 ? mp0 : q == 1 ? mp1 : mp2;
    bool inc = false;
    for (int k = 0; k < num; k++) inc |= mq == list[k];
    if (!inc) list[num++] = mq;
  }
  is.n_cand = num;
  for (int k = 0; k < 11; k++) is.cand[k] = (uint8_t)(k < num ? list[k] : 0);
  wsync();
}

// xIntraCodingTUBlock (:1088)
__device__ void intra_coding_tu(Cu *cu, Yuv *org, Yuv *pred, Yuv *resi, uint32_t *dist, int comp, const Tu &t, int save_load) {
  if (!tu_proc(t, comp)) return;
  State *S = E.S;
  const int rel = tu_abs_rel(t);
  const int w = t.w[comp], h = t.h[comp], x0 = t.x0[comp], y0 = t.y0[comp];
  const int s = ystride(comp);
  int16_t *po = yaddr(org, comp, x0, y0), *pp = yaddr(pred, comp, x0, y0), *pr = yaddr(resi, comp, x0, y0);
  const int layer = qt_layer(t.log2);
  int16_t *prq = yaddr(&S->qt_yuv[layer], comp, x0, y0);
  int16_t *coef = S->qt_coef[layer] + coff(comp) + t.off[comp];
  int mode = cu->p[rel].idir[comp ? 1 : 0];
  if (comp && mode == DM_CHROMA_IDX) mode = cu->p[rel].idir[0];
  HMC(layer >= 0 && layer < 4 && t.off[comp] >= 0 && t.off[comp] + w * h <= (comp ? 1024 : 4096), 70, t.log2, t.off[comp]);
  if (save_load != 2) {
    intra_predict_tu(cu, t, comp, mode, pp);
    HMCU(cu, 71);
    if (save_load == 1) blk_copy(S->shared_pred + coff(comp), w, pp, s, w, h);
  } else blk_copy(pp, s, S->shared_pred + coff(comp), w, w, h);
  const int sh = ilog2(w);
  for (int i = lid(); i < w * h; i += 64) {
    const int k = (i >> sh) * s + (i & (w - 1));
    pr[k] = (int16_t)(po[k] - pp[k]);
  }
  wsync();
  HMCU(cu, 72);
  estimate_bit(w, h, comp ? 1 : 0);
  HMCU(cu, 73);
  if (comp == 0) set_tridx(cu, rel, 256 >> (2 * tu_depth_total(t)), tu_depth_rel(t));
  HMCU(cu, 74);
  const int32_t abs_sum = transform_tu(cu, t, comp, pr, s, coef);
  HMCU(cu, 75);
  if (abs_sum > 0) inv_transform_tu(cu, t, comp, coef, pr, s, true);  // E.td from transform_tu
  else {
    blk_copy(coef, w, nullptr, 0, w, h);
    blk_copy(pr, s, nullptr, 0, w, h);
  }
  HMCU(cu, 76);
  const int px0 = (cu->x >> (comp ? 1 : 0)) + x0, py0 = (cu->y >> (comp ? 1 : 0)) + y0;
  for (int i = lid(); i < w * h; i += 64) {
    const int y = i >> sh, x = i & (w - 1), k = y * s + x;
    const int v = clip_pel(pp[k] + pr[k]);
    pp[k] = (int16_t)v;
    prq[k] = (int16_t)v;
    *win_at(comp, px0 + x, py0 + y) = (uint8_t)v;
  }
  wsync();
  *dist += dist_part(pp, s, po, s, w, h, comp);
}
// xStoreIntraResultQT (:1758) / xLoadIntraResultQT (:1793)
__device__ void intra_store(int comp, const Tu &t) {
  if (!tu_proc(t, comp)) return;
  State *S = E.S;
  const int layer = qt_layer(t.log2), w = t.w[comp], h = t.h[comp];
  blk_copy(S->qt_tu_coef + coff(comp), w, S->qt_coef[layer] + coff(comp) + t.off[comp], w, w, h);
  blk_copy(yaddr(&S->qt_ts_yuv, comp, t.x0[comp], t.y0[comp]), ystride(comp), yaddr(&S->qt_yuv[layer], comp, t.x0[comp], t.y0[comp]),
           ystride(comp), w, h);
}
__device__ void intra_load(const Cu *cu, int comp, const Tu &t) {
  if (!tu_proc(t, comp)) return;
  State *S = E.S;
  const int layer = qt_layer(t.log2), w = t.w[comp], h = t.h[comp], s = comp ? 1 : 0;
  blk_copy(S->qt_coef[layer] + coff(comp) + t.off[comp], w, S->qt_tu_coef + coff(comp), w, w, h);
  blk_copy(yaddr(&S->qt_yuv[layer], comp, t.x0[comp], t.y0[comp]), ystride(comp), yaddr(&S->qt_ts_yuv, comp, t.x0[comp], t.y0[comp]),
           ystride(comp), w, h);
  const int px0 = (cu->x >> s) + t.x0[comp], py0 = (cu->y >> s) + t.y0[comp], sh = ilog2(w);
  for (int i = lid(); i < w * h; i += 64) {
    const int y = i >> sh, x = i & (w - 1);
    *win_at(comp, px0 + x, py0 + y) = (uint8_t)*yaddr(&S->qt_yuv[layer], comp, t.x0[comp] + x, t.y0[comp] + y);
  }
  wsync();
}

// xEncIntraHeader (:976)
__device__ void enc_intra_header(const Cu *cu, int trd, int rel, int luma, int chroma) {
  if (luma) {
    if (rel == 0) {
      if (E.P.slice_type != I_SLICE) {
        code_skip_flag(cu, 0);
        code_pred_mode(cu, 0);
      }
      code_part_size(cu, 0, cu->depth);
    }
    if (cu->p[0].part == SIZE_2Nx2N) {
      if (rel == 0) code_intra_dir_luma(cu, 0, 0);
    } else {
      const int q = cu->nparts >> 2;
      if (trd > 0 && (rel % q) == 0) code_intra_dir_luma(cu, rel, 0);
    }
  }
  if (chroma && rel == 0) code_intra_dir_chroma(cu, rel);
}
// xEncSubdivCbfQT (:866)
template <int LV>
__device__ void enc_subdiv_cbf_qt(const Cu *cu, const Tu &t, int luma, int chroma) {
  const int rel = tu_abs_rel(t), trd = tu_depth_rel(t);
  const int trmode = cu->p[rel].tr_idx, subdiv = trmode > trd, l2 = t.log2;
  if (cu->p[0].pred == MODE_INTRA && cu->p[0].part == SIZE_NxN && trd == 0) {
  } else if (l2 > 5) {
  } else if (l2 == 2) {
  } else if (l2 == qt_min_log2(cu, rel)) {
  } else if (luma) code_subdiv(subdiv, 5 - l2);
  if (chroma)
    for (int c = 1; c < 3; c++)
      if (t.all[c] && (trd == 0 || cbf_at(&cu->p[rel], c, trd - 1))) code_qt_cbf(cu, t, c, !subdiv);
  if (subdiv) {
    if constexpr (LV < 3) {
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      do enc_subdiv_cbf_qt<LV + 1>(cu, ch, luma, chroma); while (tu_next(ch, t));
    } else HMC(false, 25, LV, 0);
  } else if (luma) code_qt_cbf(cu, t, 0, 1);
}
// xEncCoeffQT (:936) on the QT temporaries
template <int LV>
__device__ void enc_coeff_qt(const Cu *cu, const Tu &t, int comp) {
  const int rel = tu_abs_rel(t), trd = tu_depth_rel(t);
  if (cu->p[rel].tr_idx > trd) {
    if constexpr (LV < 3) {
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      do enc_coeff_qt<LV + 1>(cu, ch, comp); while (tu_next(ch, t));
    } else HMC(false, 26, LV, 0);
  } else if (tu_proc(t, comp)) {
    if (cbf_at(&cu->p[tu_abs_rel_c(t, comp)], comp, trd))
      code_coeff_nxn(cu, t, comp, E.S->qt_coef[qt_layer(t.log2)] + coff(comp) + t.off[comp]);
  }
}
template <int LV>
__device__ uint32_t intra_bits_qt(const Cu *cu, const Tu &t, int luma, int chroma) {
  reset_bits();
  enc_intra_header(cu, tu_depth_rel(t), tu_abs_rel(t), luma, chroma);
  enc_subdiv_cbf_qt<LV>(cu, t, luma, chroma);
  if (luma) enc_coeff_qt<LV>(cu, t, 0);
  if (chroma) { enc_coeff_qt<LV>(cu, t, 1); enc_coeff_qt<LV>(cu, t, 2); }
  return written_bits();
}

// xRecurIntraCodingLumaQT (:1390)
template <int LV>
__device__ void recur_intra_luma_qt(Cu *cu, Yuv *org, Yuv *pred, Yuv *resi, uint32_t *dist_y, int check_first, double *rd_cost_out,
                                    const Tu &t) {
  const int rel = tu_abs_rel(t), full_depth = tu_depth_total(t), trd = tu_depth_rel(t), l2 = t.log2;
  const int check_full = l2 <= 5;
  int check_split = l2 > qt_min_log2(cu, rel);
  if (check_first && check_full) check_split = 0;
  double single_cost = kMaxDouble;
  uint32_t single_dist = 0;
  int single_cbf = 0;
  const int check_ts = t.w[0] <= 4 && cu->p[rel].part == SIZE_NxN;
  int best_mode = 0;
  const int nparts_here = 256 >> (2 * full_depth);
  if (check_full) {
    if (check_ts) {
      cload(RD(full_depth, CI_QT_TRAFO_ROOT), E.cur);
      for (int mode = 0; mode < 2; mode++) {
        uint32_t dtmp = 0;
        double ctmp;
        if (tu_proc(t, 0)) {
          set_ts_range(cu, 0, rel, nparts_here, mode);
          HMCU(cu, 50);
          intra_coding_tu(cu, org, pred, resi, &dtmp, 0, t, mode == 0 ? 1 : 2);
          HMCU(cu, 51);
        }
        const int cbf = cbf_at(&cu->p[rel], 0, trd);
        if (mode == 1 && cbf == 0) ctmp = kMaxDouble;
        else ctmp = rd_cost(intra_bits_qt<LV>(cu, t, 1, 0), dtmp);
        if (ctmp < single_cost) {
          single_cost = ctmp;
          single_dist = dtmp;
          single_cbf = cbf;
          best_mode = mode;
          if (best_mode == 0) {
            intra_store(0, t);
            cload(RD(full_depth, CI_TEMP_BEST), E.cur);
          }
        }
        if (mode == 0) cload(E.cur, RD(full_depth, CI_QT_TRAFO_ROOT));
      }
      if (tu_proc(t, 0)) set_ts_range(cu, 0, rel, nparts_here, best_mode);
      if (best_mode == 0) {
        intra_load(cu, 0, t);
        if (tu_proc(t, 0)) set_cbf_range(cu, 0, rel, nparts_here, single_cbf << trd);
        cload(E.cur, RD(full_depth, CI_TEMP_BEST));
      }
    } else {
      if (check_split) cload(RD(full_depth, CI_QT_TRAFO_ROOT), E.cur);
      if (tu_proc(t, 0)) set_ts_range(cu, 0, rel, nparts_here, 0);
      HMCU(cu, 52);
      intra_coding_tu(cu, org, pred, resi, &single_dist, 0, t, 0);
      HMCU(cu, 53);
      if (check_split) single_cbf = cbf_at(&cu->p[rel], 0, trd);
      single_cost = rd_cost(intra_bits_qt<LV>(cu, t, 1, 0), single_dist);
    }
  }
  if (check_split) {
    if constexpr (LV < 3) {
      if (check_full) {
        cload(RD(full_depth, CI_QT_TRAFO_TEST), E.cur);
        cload(E.cur, RD(full_depth, CI_QT_TRAFO_ROOT));
      } else cload(RD(full_depth, CI_QT_TRAFO_ROOT), E.cur);
      double split_cost = 0.0;
      uint32_t split_dist = 0;
      int split_cbf = 0;
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      do {
        recur_intra_luma_qt<LV + 1>(cu, org, pred, resi, &split_dist, check_first, &split_cost, ch);
        split_cbf |= cbf_at(&cu->p[tu_abs_rel(ch)], 0, tu_depth_rel(ch));
      } while (tu_next(ch, t));
      if (split_cbf) or_cbf_range(cu, 0, rel, t.step, 1 << trd);
      cload(E.cur, RD(full_depth, CI_QT_TRAFO_ROOT));
      HMCU(cu, 54);
      split_cost = rd_cost(intra_bits_qt<LV>(cu, t, 1, 0), split_dist);
      HMCU(cu, 55);
      if (split_cost < single_cost) {
        *dist_y += split_dist;
        *rd_cost_out += split_cost;
        return;
      }
      cload(E.cur, RD(full_depth, CI_QT_TRAFO_TEST));
      set_tridx(cu, rel, nparts_here, trd);
      set_cbf_range(cu, 0, rel, nparts_here, single_cbf << trd);
      set_ts_range(cu, 0, rel, nparts_here, best_mode);
      const int layer = qt_layer(l2), w = t.w[0], sh = ilog2(w);
      const int px0 = cu->x + t.x0[0], py0 = cu->y + t.y0[0];
      for (int i = lid(); i < w * w; i += 64) {
        const int y = i >> sh, x = i & (w - 1);
        *win_at(0, px0 + x, py0 + y) = (uint8_t)*yaddr(&E.S->qt_yuv[layer], 0, t.x0[0] + x, t.y0[0] + y);
      }
      wsync();
    } else HMC(false, 27, LV, 0);
  }
  *dist_y += single_dist;
  *rd_cost_out += single_cost;
}
// xSetIntraResultLumaQT (:1715)
template <int LV>
__device__ void set_intra_result_luma(Cu *cu, Yuv *reco, const Tu &t) {
  const int rel = tu_abs_rel(t);
  if (cu->p[rel].tr_idx == tu_depth_rel(t)) {
    const int layer = qt_layer(t.log2), w = t.w[0];
    if (w) {
      blk_copy(cu->coef + t.off[0], w, E.S->qt_coef[layer] + t.off[0], w, w, w);
      blk_copy(yaddr(reco, 0, t.x0[0], t.y0[0]), ystride(0), yaddr(&E.S->qt_yuv[layer], 0, t.x0[0], t.y0[0]), ystride(0), w, w);
    }
  } else {
    if constexpr (LV < 3) {
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      do set_intra_result_luma<LV + 1>(cu, reco, ch); while (tu_next(ch, t));
    } else HMC(false, 28, LV, 0);
  }
}
__device__ void save_tu_fields(Cu *cu, int poff, int np) {
  State *S = E.S;
  for (int i = lid(); i < np; i += 64) {
    const Part &p = cu->p[poff + i];
    S->tmp_tridx[i] = (uint8_t)p.tr_idx;
    for (int k = 0; k < 3; k++) { S->tmp_cbf[k][i] = p.cbf[k]; S->tmp_ts[k][i] = p.ts[k]; }
  }
  wsync();
}
__device__ void est_intra_pred_luma_qt(Cu *cu, Yuv *org, Yuv *pred, Yuv *resi, Yuv *reco) {
  State *S = E.S;
  const int depth = cu->depth;
  const int init_trd = cu->p[0].part == SIZE_2Nx2N ? 0 : 1;
  const int qnp = cu->nparts >> 2;
  uint32_t overall_dist = 0;
  for (int i = lid(); i < cu->nparts; i += 64) cu->p[i].qp = (int8_t)E.slice_qp;
  wsync();
  TU_LOCAL(tcu);
  TU_LOCAL(tpu);
  tu_root(tcu, cu, 0);
  if (init_trd) tu_child(tpu, tcu, 0);
  else tpu = tcu;
  do {
    const int poff = tu_abs_rel(tpu);
    const int n = tpu.w[0];
    HMCU(cu, 40);
    intra_first_pass(cu, tpu, org, depth);
    HMCU(cu, 41);
    HM_STAGE(2);
    if (HM_STOPPED) return;
    const int nfull = E.u.in.n_cand;
    uint8_t cand[11];
    for (int k = 0; k < 11; k++) cand[k] = E.u.in.cand[k];
    int best_mode = 0;
    uint32_t best_dist = 0;
    double best_cost = kMaxDouble;
    const int np_pu = tu_nparts(tpu, 0);
    for (int m = 0; m < nfull; m++) {
      const int mode = cand[m];
      set_idir(cu, 0, poff, np_pu, mode);
      E.cur = GOON;
      cload(E.cur, RD(depth, CI_CURR_BEST));
      uint32_t d = 0;
      double c = 0.0;
      if (init_trd) recur_intra_luma_qt<1>(cu, org, pred, resi, &d, 1, &c, tpu);
      else recur_intra_luma_qt<0>(cu, org, pred, resi, &d, 1, &c, tpu);
      HMCU(cu, 42);
      if (c < best_cost) {
        best_mode = mode; best_dist = d; best_cost = c;
        if (init_trd) set_intra_result_luma<1>(cu, reco, tpu);
        else set_intra_result_luma<0>(cu, reco, tpu);
        HMCU(cu, 43);
        save_tu_fields(cu, poff, np_pu);
        HMCU(cu, 44);
      }
    }
    {
      const int mode = best_mode;
      set_idir(cu, 0, poff, np_pu, mode);
      cload(E.cur, RD(depth, CI_CURR_BEST));
      uint32_t d = 0;
      double c = 0.0;
      if (init_trd) recur_intra_luma_qt<1>(cu, org, pred, resi, &d, 0, &c, tpu);
      else recur_intra_luma_qt<0>(cu, org, pred, resi, &d, 0, &c, tpu);
      if (c < best_cost) {
        best_mode = mode; best_dist = d; best_cost = c;
        if (init_trd) set_intra_result_luma<1>(cu, reco, tpu);
        else set_intra_result_luma<0>(cu, reco, tpu);
        save_tu_fields(cu, poff, np_pu);
      }
    }
    HMCU(cu, 45);
    overall_dist += best_dist;
    for (int i = lid(); i < np_pu; i += 64) {
      Part &p = cu->p[poff + i];
      p.tr_idx = (int8_t)S->tmp_tridx[i];
      for (int k = 0; k < 3; k++) { p.cbf[k] = S->tmp_cbf[k][i]; p.ts[k] = S->tmp_ts[k][i]; }
    }
    wsync();
    if (init_trd && tpu.section < 3) {
      const int sh = ilog2(n);
      for (int i = lid(); i < n * n; i += 64) {
        const int y = i >> sh, x = i & (n - 1);
        *win_at(0, cu->x + tpu.x0[0] + x, cu->y + tpu.y0[0] + y) = (uint8_t)*yaddr(reco, 0, tpu.x0[0] + x, tpu.y0[0] + y);
      }
      wsync();
    }
    HMCU(cu, 46);
    set_idir(cu, 0, poff, np_pu, best_mode);
    HMCU(cu, 47);
  } while (init_trd && tu_next(tpu, tcu));
  if (init_trd) {
    int cy = 0, cb = 0, cr = 0;
    for (int p = 0; p < 4; p++) {
      cy |= cbf_at(&cu->p[p * qnp], 0, 1);
      cb |= cbf_at(&cu->p[p * qnp], 1, 1);
      cr |= cbf_at(&cu->p[p * qnp], 2, 1);
    }
    for (int i = lid(); i < 4 * qnp; i += 64) { cu->p[i].cbf[0] |= (uint8_t)cy; cu->p[i].cbf[1] |= (uint8_t)cb; cu->p[i].cbf[2] |= (uint8_t)cr; }
    wsync();
  }
  HMCU(cu, 48);
  cload(E.cur, RD(depth, CI_CURR_BEST));
  cu->dist = overall_dist;
}

// xRecurIntraChromaCodingQT (:1913)
template <int LV>
__device__ void recur_intra_chroma_qt(Cu *cu, Yuv *org, Yuv *pred, Yuv *resi, uint32_t *dist, const Tu &t) {
  const int rel = tu_abs_rel(t), trd = tu_depth_rel(t);
  const int trmode = cu->p[rel].tr_idx;
  if (trmode == trd) {
    if (!tu_proc(t, 1)) return;
    const int full_depth = tu_depth_total(t);
    int check_ts = t.w[1] <= 4;
    if (check_ts) {
      check_ts &= t.w[0] <= 4;
      if (check_ts) {
        int nb = 0;
        const int maxp = rel + (t.all[1] ? 1 : 4);
        for (int i = rel; i < maxp; i++) nb += cu->p[i].ts[0];
        check_ts &= nb > 0;
      }
    }
    for (int c = 1; c < 3; c++) {
      cload(RD(full_depth, CI_QT_TRAFO_ROOT), E.cur);
      const int crel = tu_abs_rel_c(t, c), np = tu_nparts(t, c);
      double single_cost = kMaxDouble;
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
        intra_coding_tu(cu, org, pred, resi, &dtmp, c, t, sl);
        const int cbf = cbf_at(&cu->p[crel], c, trd);
        if (tsm == 1 && cbf == 0) ctmp = kMaxDouble;
        else if (!one) {
          reset_bits();
          enc_coeff_qt<LV>(cu, t, c);
          ctmp = rd_cost(written_bits(), dtmp);
        }
        if (ctmp < single_cost) {
          single_cost = ctmp; single_dist = dtmp; best_ts = tsm; best_id = cur_id; single_cbf = cbf;
          if (!one && !last) {
            intra_store(c, t);
            cload(RD(full_depth, CI_TEMP_BEST), E.cur);
          }
        }
        if (!one && !last) cload(E.cur, RD(full_depth, CI_QT_TRAFO_ROOT));
      }
      if (best_id < total) {
        intra_load(cu, c, t);
        set_cbf_range(cu, c, crel, np, single_cbf << trd);
        cload(E.cur, RD(full_depth, CI_TEMP_BEST));
      }
      set_ts_range(cu, c, crel, np, best_ts);
      *dist += single_dist;
    }
  } else {
    if constexpr (LV < 3) {
      int scb = 0, scr = 0;
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      const int trd_child = tu_depth_rel(ch);
      do {
        recur_intra_chroma_qt<LV + 1>(cu, org, pred, resi, dist, ch);
        const int sub = tu_abs_rel(ch);
        scb |= cbf_at(&cu->p[sub], 1, trd_child);
        scr |= cbf_at(&cu->p[sub], 2, trd_child);
      } while (tu_next(ch, t));
      if (scb) or_cbf_range(cu, 1, rel, t.step, 1 << trd);
      if (scr) or_cbf_range(cu, 2, rel, t.step, 1 << trd);
    } else HMC(false, 29, LV, 0);
  }
}
// xSetIntraResultChromaQT (:2124)
template <int LV>
__device__ void set_intra_result_chroma(Cu *cu, Yuv *reco, const Tu &t) {
  if (!tu_proc(t, 1)) return;
  const int rel = tu_abs_rel(t);
  if (cu->p[rel].tr_idx == tu_depth_rel(t)) {
    const int layer = qt_layer(t.log2), w = t.w[1];
    for (int c = 1; c < 3; c++) {
      blk_copy(cu->coef + coff(c) + t.off[c], w, E.S->qt_coef[layer] + coff(c) + t.off[c], w, w, w);
      blk_copy(yaddr(reco, c, t.x0[c], t.y0[c]), ystride(c), yaddr(&E.S->qt_yuv[layer], c, t.x0[c], t.y0[c]), ystride(c), w, w);
    }
  } else {
    if constexpr (LV < 3) {
      TU_LOCAL(ch);
      tu_child(ch, t, 0);
      do set_intra_result_chroma<LV + 1>(cu, reco, ch); while (tu_next(ch, t));
    } else HMC(false, 30, LV, 0);
  }
}
__device__ void est_intra_pred_chroma_qt(Cu *cu, Yuv *org, Yuv *pred, Yuv *resi, Yuv *reco) {
  State *S = E.S;
  const int depth = cu->depth;
  TU_LOCAL(t);
  tu_root(t, cu, 0);
  const int np = t.step;
  int best_mode = 0;
  uint32_t best_dist = 0;
  double best_cost = kMaxDouble;
  int m0 = 0, m1 = 26, m2 = 10, m3 = 1;
  const int lm = cu->p[0].idir[0];
  if (lm == m0) m0 = 34;
  else if (lm == m1) m1 = 34;
  else if (lm == m2) m2 = 34;
  else if (lm == m3) m3 = 34;
  for (int m = 0; m < 5; m++) {
    const int mode = m == 0 ? m0 : m == 1 ? m1 : m == 2 ? m2 : m == 3 ? m3 : DM_CHROMA_IDX;
    E.cur = GOON;
    cload(E.cur, RD(depth, CI_CURR_BEST));
    uint32_t d = 0;
    set_idir(cu, 1, 0, np, mode);
    recur_intra_chroma_qt<0>(cu, org, pred, resi, &d, t);
    cload(E.cur, RD(depth, CI_CURR_BEST));
    const uint32_t b = intra_bits_qt<0>(cu, t, 0, 1);
    const double c = rd_cost(b, d);
    if (c < best_cost) {
      best_cost = c; best_dist = d; best_mode = mode;
      set_intra_result_chroma<0>(cu, reco, t);
      for (int i = lid(); i < np; i += 64)
        for (int k = 1; k < 3; k++) { S->save_cbf[k][i] = cu->p[i].cbf[k]; S->save_ts[k][i] = cu->p[i].ts[k]; }
      wsync();
    }
  }
  for (int i = lid(); i < np; i += 64)
    for (int k = 1; k < 3; k++) { cu->p[i].cbf[k] = S->save_cbf[k][i]; cu->p[i].ts[k] = S->save_ts[k][i]; }
  wsync();
  set_idir(cu, 1, 0, np, best_mode);
  cu->dist += best_dist;
  cload(E.cur, RD(depth, CI_CURR_BEST));
}

// ============================================================================================
// TEncCu: xCheckBestMode (:1444), xCheckRDCostMerge2Nx2N (:1166), xCheckRDCostInter (:1291),
// xCheckRDCostIntra (:1330), deriveTestModeAMP (:274), xCompressCU (:349)
// ============================================================================================
__device__ void check_best_mode(int depth) {
  const double tc = TEMP(depth)->cost, bc = BEST(depth)->cost;
  if (tc < bc) {
    wsync();
    int t = E.best[depth]; E.best[depth] = E.temp[depth]; E.temp[depth] = t;
    t = E.yi[Y_PRED_BEST][depth]; E.yi[Y_PRED_BEST][depth] = E.yi[Y_PRED_TEMP][depth]; E.yi[Y_PRED_TEMP][depth] = t;
    t = E.yi[Y_RECO_BEST][depth]; E.yi[Y_RECO_BEST][depth] = E.yi[Y_RECO_TEMP][depth]; E.yi[Y_RECO_TEMP][depth] = t;
    wsync();
    cload(RD(depth, CI_NEXT_BEST), RD(depth, CI_TEMP_BEST));
  }
}
__device__ __forceinline__ void reinit_temp(int depth) { cu_init_est(TEMP(depth), E.slice_qp); }

__device__ void check_rd_merge2nx2n(int depth) {
  cu_set_all(TEMP(depth), F_PART, SIZE_2Nx2N);
  MergeList m;
  merge_candidates(TEMP(depth), SIZE_2Nx2N, 0, m);
  const int n = m.n;
  int buf = 0;  // mergeCandBuffer bits
  int best_is_skip = 0;
  for (int nores = 0; nores < 2; nores++) {
    for (int k = 0; k < n; k++) {
      if (nores == 1 && ((buf >> k) & 1)) continue;
      if (best_is_skip && nores == 0) continue;
      Cu *tmp = TEMP(depth);
      const int np = tmp->nparts;
      const MvField f0 = m.f[2 * k], f1 = m.f[2 * k + 1];
      const int dir = m.dirs[k];
      for (int i = lid(); i < np; i += 64) {
        Part &p = tmp->p[i];
        p.pred = MODE_INTER;
        p.part = SIZE_2Nx2N;
        p.merge = 1;
        p.merge_idx = (int8_t)k;
        p.inter_dir = (int8_t)dir;
        p.mv[0][0] = f0.mv[0]; p.mv[0][1] = f0.mv[1]; p.ref[0] = (int8_t)f0.ref;
        p.mv[1][0] = f1.mv[0]; p.mv[1][1] = f1.mv[1]; p.ref[1] = (int8_t)f1.ref;
      }
      wsync();
      mc_cu(tmp, YB(Y_PRED_TEMP, depth));
      enc_res_rd_inter(tmp, YB(Y_ORIG, depth), YB(Y_PRED_TEMP, depth), YB(Y_RESI_TEMP, depth), YB(Y_RESI_BEST, depth),
                       YB(Y_RECO_TEMP, depth), nores != 0);
      if (nores == 0 && !cu_qt_root_cbf(tmp, 0)) buf |= 1 << k;
      check_best_mode(depth);
      reinit_temp(depth);
      if (!best_is_skip) best_is_skip = !cu_qt_root_cbf(BEST(depth), 0);
    }
  }
}
__device__ void check_rd_inter(int depth, int ps, int use_mrg) {
  Cu *tmp = TEMP(depth);
  cu_set_all(tmp, F_PART, ps);
  cu_set_all(tmp, F_PRED, MODE_INTER);
  tmp->merge_amp = 1;
  pred_inter_search(tmp, YB(Y_ORIG, depth), YB(Y_PRED_TEMP, depth), use_mrg);
  enc_res_rd_inter(tmp, YB(Y_ORIG, depth), YB(Y_PRED_TEMP, depth), YB(Y_RESI_TEMP, depth), YB(Y_RESI_BEST, depth),
                   YB(Y_RECO_TEMP, depth), 0);
  const double c = cu_cost(tmp->dssim, tmp->bits, tmp->dist);
  wsync();
  tmp->cost = c;
  check_best_mode(depth);
}
__device__ void check_rd_intra(int depth, int ps) {
  if (HM_STOPPED) return;
  Cu *tmp = TEMP(depth);
  cu_set_all(tmp, F_SKIP, 0);
  cu_set_all(tmp, F_PART, ps);
  cu_set_all(tmp, F_PRED, MODE_INTRA);
  HMCU(tmp, 62);
  est_intra_pred_luma_qt(tmp, YB(Y_ORIG, depth), YB(Y_PRED_TEMP, depth), YB(Y_RESI_TEMP, depth), YB(Y_RECO_TEMP, depth));
  HMCU(tmp, 60);
  HM_STAGE(3);
  if (HM_STOPPED) return;
  yuv_to_pic_comp(YB(Y_RECO_TEMP, depth), tmp, 0);
  HMCU(tmp, 61);
  est_intra_pred_chroma_qt(tmp, YB(Y_ORIG, depth), YB(Y_PRED_TEMP, depth), YB(Y_RESI_TEMP, depth), YB(Y_RECO_TEMP, depth));
  HM_STAGE(4);
  if (HM_STOPPED) return;
  reset_bits();
  code_skip_flag(tmp, 0);
  code_pred_mode(tmp, 0);
  code_part_size(tmp, 0, depth);
  encode_pred_info(tmp, 0);
  encode_coeff(tmp, 0);
  cload(RD(depth, CI_TEMP_BEST), E.cur);
  const uint32_t b = written_bits();
  const double c = cu_cost(measure_ssim(tmp, YB(Y_ORIG, depth), YB(Y_RECO_TEMP, depth)), b, tmp->dist);
  tmp->bits = b;
  tmp->cost = c;
  check_best_mode(depth);
}
__device__ void derive_test_mode_amp(const Cu *best, int parent_ps, int &hor, int &ver, int &mhor, int &mver) {
  const int ps = best->p[0].part;
  if (ps == SIZE_2NxN) hor = 1;
  else if (ps == SIZE_Nx2N) ver = 1;
  else if (ps == SIZE_2Nx2N && !best->p[0].merge && !best->p[0].skip) { hor = 1; ver = 1; }
  if (parent_ps >= SIZE_2NxnU && parent_ps <= SIZE_nRx2N) { mhor = 1; mver = 1; }
  if (parent_ps == SIZE_NONE) {
    if (ps == SIZE_2NxN) mhor = 1;
    else if (ps == SIZE_Nx2N) mver = 1;
  }
  if (ps == SIZE_2Nx2N && !best->p[0].skip) { mhor = 1; mver = 1; }
  if (best->width == 64) { hor = 0; ver = 0; }
}

template <int D>
__device__ void compress_cu(int parent_ps) {
  if (HM_STOPPED) return;
  const int depth = D;
  E.yw = 64 >> D;
  Cu *best = BEST(depth);
  if (lid() == 0) E.S->rq_n[D] = 0;  // the inter residual memo holds this CU's RQTs only
  copy_org_to_yuv(YB(Y_ORIG, depth), best);
  int boundary = 0;
  const int rx = best->x + best->width - 1, by = best->y + best->width - 1;
  const int qp = E.slice_qp;
  if (rx < E.P.w && by < E.P.h) {
    reinit_temp(depth);
    if (E.P.slice_type != I_SLICE) {
      check_rd_merge2nx2n(depth);
      reinit_temp(depth);
      check_rd_inter(depth, SIZE_2Nx2N, 0);
      reinit_temp(depth);
    }
    reinit_temp(depth);
    if (E.P.slice_type != I_SLICE) {
      check_rd_inter(depth, SIZE_Nx2N, 0);
      reinit_temp(depth);
      check_rd_inter(depth, SIZE_2NxN, 0);
      reinit_temp(depth);
      if (E.P.amp && depth < 3) {
        int hor = 0, ver = 0, mhor = 0, mver = 0;
        derive_test_mode_amp(BEST(depth), parent_ps, hor, ver, mhor, mver);
        if (hor) {
          check_rd_inter(depth, SIZE_2NxnU, 0); reinit_temp(depth);
          check_rd_inter(depth, SIZE_2NxnD, 0); reinit_temp(depth);
        } else if (mhor) {
          check_rd_inter(depth, SIZE_2NxnU, 1); reinit_temp(depth);
          check_rd_inter(depth, SIZE_2NxnD, 1); reinit_temp(depth);
        }
        if (ver) {
          check_rd_inter(depth, SIZE_nLx2N, 0); reinit_temp(depth);
          check_rd_inter(depth, SIZE_nRx2N, 0); reinit_temp(depth);
        } else if (mver) {
          check_rd_inter(depth, SIZE_nLx2N, 1); reinit_temp(depth);
          check_rd_inter(depth, SIZE_nRx2N, 1); reinit_temp(depth);
        }
      }
    }
    best = BEST(depth);
    if (E.P.slice_type == I_SLICE || (best->p[0].cbf[0] || best->p[0].cbf[1] || best->p[0].cbf[2])) {
      check_rd_intra(depth, SIZE_2Nx2N);
      reinit_temp(depth);
      if (depth == 3 && TEMP(depth)->width > 4) {
        check_rd_intra(depth, SIZE_NxN);
        reinit_temp(depth);
      }
    }
    best = BEST(depth);
    E.cur = GOON;
    cload(E.cur, RD(depth, CI_NEXT_BEST));
    reset_bits();
    code_split_flag(best, 0, depth);
    const uint32_t b = best->bits + written_bits();
    const double c = cu_cost(best->dssim, b, best->dist);
    wsync();
    best->bits = b;
    best->cost = c;
    cload(RD(depth, CI_NEXT_BEST), E.cur);
  } else boundary = 1;

  reinit_temp(depth);
  if constexpr (D < 3) {
    const int nd = depth + 1;
    for (int k = 0; k < 4; k++) {
      cu_init_sub(BEST(nd), TEMP(depth), k, nd, qp);
      cu_init_sub(TEMP(nd), TEMP(depth), k, nd, qp);
      Cu *sb = BEST(nd);
      if (sb->x < E.P.w && sb->y < E.P.h) {
        if (k == 0) cload(RD(nd, CI_CURR_BEST), RD(depth, CI_CURR_BEST));
        else cload(RD(nd, CI_CURR_BEST), RD(nd, CI_NEXT_BEST));
        const int pps = BEST(depth)->p[0].pred != MODE_INTER ? SIZE_NONE : BEST(depth)->p[0].part;
        compress_cu<D + 1>(pps);
        cu_copy_part_from(TEMP(depth), BEST(nd), k, nd);
        yuv_child_to_parent(YB(Y_RECO_TEMP, depth), YB(Y_RECO_BEST, nd), k, 64 >> nd);
      } else {
        cu_copy_to_pic(sb);
        cu_copy_part_from(TEMP(depth), sb, k, nd);
      }
    }
    E.yw = 64 >> D;  // the children left their own layout
    Cu *tmp = TEMP(depth);
    E.cur = GOON;
    cload(E.cur, RD(nd, CI_NEXT_BEST));
    uint32_t b = tmp->bits;
    if (!boundary) {
      reset_bits();
      code_split_flag(tmp, 0, depth);
      b += written_bits();
    }
    const double c = cu_cost(tmp->dssim, b, tmp->dist);
    wsync();
    tmp->bits = b;
    tmp->cost = c;
    cload(RD(depth, CI_TEMP_BEST), E.cur);
    check_best_mode(depth);
  }
  cu_copy_to_pic(BEST(depth));
  yuv_to_pic(YB(Y_RECO_BEST, depth), BEST(depth));
}

// ============================================================================================
// TEncCu::xEncodeCU (:920) under the counter: the CTU coding whose states start the next CTU
// ============================================================================================
template <int D>
__device__ void encode_cu(int rel, int last_ctu_in_slice) {
  const int depth = D;
  State *S = E.S;
  const int r = z2r(rel);
  const int lx = E.ctu_x * 64 + rpx(r), ty = E.ctu_y * 64 + rpy(r);
  const int sz = 64 >> depth;
  const int rx = lx + sz - 1, by = ty + sz - 1;
  Cu *ctu = &S->view;  // depth-0 view of the CTU (zidx 0)
  int boundary = 0;
  if (rx < E.P.w && by < E.P.h) code_split_flag(ctu, rel, depth);
  else boundary = 1;
  if ((depth < ctu->p[rel].depth && depth < 3) || boundary) {
    if constexpr (D < 3) {
      const int q = (256 >> (2 * depth)) >> 2;
      for (int k = 0; k < 4; k++) {
        const int sub = rel + k * q, rs = z2r(sub);
        if (E.ctu_x * 64 + rpx(rs) < E.P.w && E.ctu_y * 64 + rpy(rs) < E.P.h) encode_cu<D + 1>(sub, last_ctu_in_slice);
      }
    } else HMC(false, 31, D, 0);
    return;
  }
  code_skip_flag(ctu, rel);
  if (ctu->p[rel].skip) {
    code_merge_index(ctu, rel);
  } else {
    code_pred_mode(ctu, rel);
    code_part_size(ctu, rel, depth);
    encode_pred_info(ctu, rel);
    if (ctu->p[rel].pred != MODE_INTRA && !(ctu->p[rel].merge && ctu->p[rel].part == SIZE_2Nx2N))
      cbin(X_ROOT_CBF, cu_qt_root_cbf(ctu, rel));
    if (ctu->p[rel].pred == MODE_INTRA || cu_qt_root_cbf(ctu, rel)) {
      // TComTURecurse(pcCU, uiAbsPartIdx, uiDepth) over the CTU: a CU-relative view (the decision
      // is over, so a temp CU object serves as its storage)
      Cu *view = &S->cu[E.temp[0]];
      const int np = 256 >> (2 * depth), off = rel * 16;
      wsync();
      view->depth = depth; view->zidx = rel; view->width = sz; view->nparts = np;
      view->x = lx; view->y = ty;
      copy_words(view->p, &ctu->p[rel], (int)sizeof(Part) * np);
      copy_words(view->coef, ctu->coef + off, 2 * sz * sz);
      copy_words(view->coef + 4096, ctu->coef + 4096 + (off >> 2), sz * sz >> 1);
      copy_words(view->coef + 5120, ctu->coef + 5120 + (off >> 2), sz * sz >> 1);
      wsync();
      TU_LOCAL(t);
      tu_root(t, view, 0);
      encode_transform<0>(view, t);
    }
  }
  const int ex = lx + sz, ey = ty + sz;
  if ((ex % 64 == 0 || ex == E.P.w) && (ey % 64 == 0 || ey == E.P.h) && !last_ctu_in_slice) ctrm(0);
}

// ============================================================================================
// compressCtu of one CTU (initCtu, the decision, then encodeCtu on the entry coder)
// ============================================================================================
__device__ void compress_ctu(int addr, const Coder *entry_g, int entry_in_lds, Coder *after_g) {
  State *S = E.S;
  E.ctu_addr = addr;
  E.ctu_x = addr % E.P.w_ctus;
  E.ctu_y = addr / E.P.w_ctus;
  E.slice_qp = E.P.qp;
  for (int d = 0; d < 4; d++) {
    E.best[d] = d;
    E.temp[d] = 4 + d;
    for (int k = 0; k < 7; k++) E.yi[k][d] = k * 4 + d;
  }
  // estBits start from zero per CTU like the restatement (every table entry RDOQ reads is
  // rewritten by estimateBit before its first use)
  for (int i = lid(); i < (int)(sizeof(hvx_estbits) / 4); i += 64) ((uint32_t *)&E.est)[i] = 0;
  if (lid() == 0) E.est_key = 0;
  wsync();
  // initCtu of the picture's CTU and the depth-0 best/temp CUs
  for (int k = 0; k < 2; k++) {
    Cu *c = &S->cu[k * 4];
    c->depth = 0; c->width = 64; c->nparts = 256; c->zidx = 0;
    c->x = E.ctu_x * 64; c->y = E.ctu_y * 64;
    cu_init_est(c, E.P.qp);
  }
  copy_words(S->ctu_p, S->cu[0].p, (int)sizeof(Part) * 256);
  for (int i = lid(); i < 3072; i += 64) ((uint32_t *)S->ctu_coef)[i] = 0;
  for (int i = lid(); i < 1536; i += 64) ((uint32_t *)S->win)[i] = 0;
  wsync();
  S->ctu_bits = 0; S->ctu_dist = 0; S->ctu_cost = kMaxDouble;
  // m_pppcRDSbacCoder[0][CI_CURR_BEST] <- the entry state
  Coder &c0 = E.cod[RD(0, CI_CURR_BEST)];
  if (!entry_in_lds) {
    copy_words(&c0, entry_g, (int)sizeof(Coder));
    wsync();
  }
  E.cur = GOON;
  cload(E.cur, RD(0, CI_CURR_BEST));  // TEncSlice.cpp:764
  // the entry state aside for encodeCtu (CI_CHROMA_INTRA coders are never used by the decision)
  cload(RD(5, CI_CHROMA_INTRA), RD(0, CI_CURR_BEST));
  HM_STAGE(1);
  {
    HM_PROF(PR_CTU);
    compress_cu<0>(SIZE_NONE);
  }
  HM_STAGE(5);
  if (HM_STOPPED) return;
  // encodeCtu on m_pppcRDSbacCoder[0][CI_CURR_BEST] after resetBits (TEncSlice.cpp:821-828)
  E.cur = RD(0, CI_CURR_BEST);
  cload(E.cur, RD(5, CI_CHROMA_INTRA));
  reset_bits();
  Cu *v = &S->view;
  wsync();
  v->depth = 0; v->zidx = 0; v->width = 64; v->nparts = 256;
  v->x = E.ctu_x * 64; v->y = E.ctu_y * 64;
  copy_words(v->p, S->ctu_p, (int)sizeof(Part) * 256);
  copy_words(v->coef, S->ctu_coef, 2 * 6144);
  wsync();
  {
    HM_PROF(PR_ENC);
    encode_cu<0>(0, addr == E.slice_end);
  }
  if (after_g) {
    copy_words(after_g, &E.cod[E.cur], (int)sizeof(Coder));
    wsync();
  }
}
#undef E
}  // namespace hm

// hvx_hm_compress: one workgroup (one wave) per job
#ifdef HM_WAVES_PER_EU
#define HM_KATTR __attribute__((amdgpu_waves_per_eu(HM_WAVES_PER_EU)))
#else
#define HM_KATTR
#endif
// the preconditions of a job (include/hvx.h hvx_hm_compress): 0 when it may run, else the
// HVX_HM_BAD_* code of the first violated one (the job is then skipped: nothing is written)
__device__ int hm_job_check(const hvx_hm_picture *pics, int n_pics, const hvx_hm_job &j, int n_out) {
  if (j.pic < 0 || j.pic >= n_pics) return HVX_HM_BAD_PIC;
  const hvx_hm_picture &P = pics[j.pic];
  if (P.w <= 0 || P.h <= 0 || (P.w & 7) || (P.h & 7) || P.w_ctus != (P.w + 63) / 64 || P.h_ctus != (P.h + 63) / 64)
    return HVX_HM_BAD_GEOMETRY;
  if (P.slice_type < 0 || P.slice_type > 2 || P.nref[0] < 0 || P.nref[0] > 4 || P.nref[1] < 0 || P.nref[1] > 4 ||
      (P.slice_type != 0 && P.nref[1] != 0) || (P.slice_type == 2 && P.nref[0] != 0) || (P.slice_type != 2 && P.nref[0] < 1))
    return HVX_HM_BAD_REFS;
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < P.nref[l]; i++) {
      const int k = P.ref_plane[l][i];
      if (k < 0 || k >= 8 || !P.ref8[k] || !P.ref16[k][0] || !P.ref16[k][1] || !P.ref16[k][2]) return HVX_HM_BAD_REFS;
    }
  if (!P.org[0] || !P.org[1] || !P.org[2] || !P.rec[0] || !P.rec[1] || !P.rec[2] || !P.ctus || !P.entropy_bits ||
      (P.col_valid && !P.col_field))
    return HVX_HM_BAD_PLANES;
  const int n = P.w_ctus * P.h_ctus;
  if (j.first_ctu < 0 || j.n_ctus < 1 || j.first_ctu + j.n_ctus > n) return HVX_HM_BAD_CTUS;
  if (HVX_HM_SLICE_CTUS_OF(j.flags) == 0 &&
      (j.slice_start < 0 || j.slice_start > j.first_ctu || j.slice_end < j.first_ctu + j.n_ctus - 1 || j.slice_end >= n))
    return HVX_HM_BAD_CTUS;
  if (j.out < 0 || (n_out > 0 && j.out + j.n_ctus > n_out)) return HVX_HM_BAD_OUT;
  return 0;
}

static __global__ __launch_bounds__(64) HM_KATTR void k_hm_compress(const hvx_hm_picture *__restrict__ pics, int n_pics,
                                                    const hvx_hm_job *__restrict__ jobs, int n_jobs, int n_out,
                                                    char *state_base, size_t state_bytes, hvx_hm_ctu *out_ctu,
                                                    uint8_t *out_rec, hvx_hm_coder *out_coder) {
  using namespace hm;
  const int jid = blockIdx.x;
  if (jid >= n_jobs) return;
  const int l = threadIdx.x;
  const hvx_hm_job &job = jobs[jid];
  State *S = (State *)(state_base + (size_t)jid * state_bytes);
  {
    const int bad = hm_job_check(pics, n_pics, job, n_out);
    if (l < 4) S->status[l] = l == 0 ? -bad : 0;  // the job's status word (hvx_hm_job_status)
    if (l < 4) S->dbg[l] = 0;
    if (bad) return;
  }
  // the wave's LDS record starts zeroed, so nothing the decision reads before writing it (every
  // such read is a bug) depends on what the previous workgroup on this CU left there
  for (int i = l; i < (int)(sizeof(Enc) / 4); i += 64) reinterpret_cast<uint32_t *>(&hm_e)[i] = 0;
  wsync();
  copy_words(&hm_e.P, &pics[job.pic], (int)sizeof(hvx_hm_picture));
  wsync();
  hm_fill_pk(hm_e.P.entropy_bits, l);
  hm_e.S = S;
  if (l < 4) hm_e.dbg[l] = 0;
  hm_e.stage = job.flags >> 8;
  hm_e.slice_start = job.slice_start;
  hm_e.slice_end = job.slice_end;
  hm_e.stop = 0;
  hm_e.tsp = 0;
#ifdef HM_PROFILE
  hm_e.prof[l >> 5][l & 31] = 0;
#endif
  const int resume = job.flags & HVX_HM_RESUME;
  if (resume) {
    copy_words(&hm_e.cod[RD(0, CI_CURR_BEST)], &S->carry, (int)sizeof(Coder));
    if (l < kMemoK) { hm_e.memo_key[l] = S->memo[l].key; hm_e.memo_hash[l] = S->memo[l].hash; }
    hm_e.memo_next = S->memo_next;
    if (l < kMemoB) { hm_e.memob_key[l] = S->memob[l].key; hm_e.memob_hash[l] = S->memob[l].hash; }
    hm_e.memob_next = S->memob_next;
  } else {
    copy_words(S->int2n, job.int2n, (int)sizeof(S->int2n));
    if (l < kMemoK) S->memo[l].key = 0;  // the count memo starts empty
    if (l == 0) S->memo_next = 0;
    if (l < kMemoK) { hm_e.memo_key[l] = 0; hm_e.memo_hash[l] = 0; }
    hm_e.memo_next = 0;
    if (l < kMemoB) { S->memob[l].key = 0; hm_e.memob_key[l] = 0; hm_e.memob_hash[l] = 0; }
    if (l == 0) S->memob_next = 0;
    hm_e.memob_next = 0;
  }
  wsync();
  const int n = job.n_ctus;
  const int slice_ctus = HVX_HM_SLICE_CTUS_OF(job.flags), nctu = hm_e.P.w_ctus * hm_e.P.h_ctus;
  for (int k = 0; k < n; k++) {
    const int addr = job.first_ctu + k;
    const int slot = job.out + k;
    // a chain over consecutive SliceMode=1 slices: each slice's first CTU starts from the slice-start
    // coder (entry) while TEncSearch's m_integerMv2Nx2N carries on, as TEncSlice::compressSlice does
    bool slice_first = false;
    if (slice_ctus > 0) {
      const int s0 = addr - addr % slice_ctus;
      wsync();
      hm_e.slice_start = s0;
      hm_e.slice_end = (s0 + slice_ctus < nctu ? s0 + slice_ctus : nctu) - 1;
      wsync();
      slice_first = addr == s0;
    }
    compress_ctu(addr, &job.entry, (k > 0 || resume) && !slice_first, out_coder ? &out_coder[slot] : nullptr);
    // the next CTU starts from this CTU's encodeCtu state (m_pppcRDSbacCoder[0][CI_CURR_BEST])
    // which compress_ctu left in coder RD(0, CI_CURR_BEST)
    copy_words(&S->carry, &hm_e.cod[RD(0, CI_CURR_BEST)], (int)sizeof(Coder));
    if (l < 4) S->dbg[l] = hm_e.dbg[l];
#ifdef HM_PROFILE
    S->prof[l >> 5][l & 31] = hm_e.prof[l >> 5][l & 31];
#endif
    hvx_hm_ctu *o = &out_ctu[slot];
    copy_words(o->p, S->ctu_p, (int)sizeof(Part) * 256);
    copy_words(o->coef, S->ctu_coef, 2 * 6144);
    {  // the window, 0 outside the picture
      uint8_t *orec = out_rec + (size_t)slot * 6144;
      for (int c = 0; c < 3; c++) {
        const int s = c ? 1 : 0, cs = 64 >> s, W = hm_e.P.w >> s, H = hm_e.P.h >> s;
        for (int i = l; i < cs * cs; i += 64) {
          const int y = i / cs, x = i - y * cs;
          const bool in = hm_e.ctu_x * cs + x < W && hm_e.ctu_y * cs + y < H;
          orec[coff(c) + i] = in ? S->win[coff(c) + i] : 0;
        }
      }
    }
    wsync();
    if (l == 0) { o->bits = S->ctu_bits; o->dist = S->ctu_dist; o->cost = S->ctu_cost; }
    if (job.chained) {
      hvx_hm_ctu *pc = &hm_e.P.ctus[addr];
      copy_words(pc->p, S->ctu_p, (int)sizeof(Part) * 256);
      copy_words(pc->coef, S->ctu_coef, 2 * 6144);
      if (l == 0) { pc->bits = S->ctu_bits; pc->dist = S->ctu_dist; pc->cost = S->ctu_cost; }
      const int cx = hm_e.ctu_x, cy = hm_e.ctu_y;
      for (int c = 0; c < 3; c++) {
        const int s = c ? 1 : 0, cs = 64 >> s, W = hm_e.P.w >> s, H = hm_e.P.h >> s, rs = hm_e.P.rec_stride[s];
        uint8_t *dst = hm_e.P.rec[c];
        for (int i = l; i < cs * cs; i += 64) {
          const int y = i / cs, x = i - y * cs, px = cx * cs + x, py = cy * cs + y;
          if (px < W && py < H) dst[py * rs + px] = S->win[coff(c) + y * cs + x];
        }
      }
      __threadfence();
      wsync();
    }
  }
}

/* stv_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Calls the reference stvssim.c metric functions (compiled unmodified from
 * /root/reference/stvssim_src/stvssimrdo2_att/lencod/src/stvssim.c into
 * oracle/_ref/stvssim.o) from plain arrays, for golden-vector generation.
 *
 * The JM encoder that normally hosts stvssim.c needs OpenCV 2.1 (absent), so
 * this harness provides the JM global *variables* stvssim.c reads
 * (params->SSIMOverlapSize, img->max_imgpel_value_comp) and fills the history
 * buffers refPicsData/srcPicsData/pic_directions2 the way
 * storeRefAndEncFrames / getDirection_macroblock would.  stvssim.c calls
 * `min(a,b)`, which on the original MSVC build is the <stdlib.h> macro; it is
 * supplied here with the same semantics.
 */
#include "global.h"
#include "stvssim.h"

InputParameters *params;
ImageParameters *img;
struct storable_picture *enc_picture;
void *stats;

int min(int a, int b) { return a < b ? a : b; }

double lambda_2(int qp);
double adjust_lambda(double lambda, double eta);

static InputParameters g_params;
static ImageParameters g_img;

#define HN 26
#define B 32

static imgpel **alloc2d(int h, int w) {
  imgpel **p = (imgpel **)malloc(sizeof(imgpel *) * h);
  imgpel *d = (imgpel *)calloc((size_t)h * w, sizeof(imgpel));
  for (int i = 0; i < h; i++) p[i] = d + (size_t)i * w;
  return p;
}

static void setup(int overlap) {
  params = &g_params;
  img = &g_img;
  params->SSIMOverlapSize = overlap;
  for (int c = 0; c < 3; c++) img->max_imgpel_value_comp[c] = 255;
}

float stv_compute_ssim(const unsigned char *org, const unsigned char *rec, int w, int h, int wint, int overlap, int comp) {
  setup(overlap);
  imgpel **o = alloc2d(B, B), **r = alloc2d(B, B);
  for (int y = 0; y < B; y++)
    for (int x = 0; x < B; x++) { o[y][x] = org[y * B + x]; r[y][x] = rec[y * B + x]; }
  float v = compute_SSIM(o, r, 0, 0, 0, 0, h, w, wint, comp);
  free(o[0]); free(o); free(r[0]); free(r);
  return v;
}

float stv_compute_stvssim(const unsigned char *org_hist, const unsigned char *rec_hist, const float *dirs,
                          int w, int h, int wint, int overlap, int gama, int comp,
                          float *ssim, float *ssim3d, float *stvssim) {
  setup(overlap);
  static int inited = 0;
  if (!inited) {
    for (int f = 0; f < REFNUM; f++)
      for (int c = 0; c < 3; c++) { refPicsData[f][c] = alloc2d(B, B); srcPicsData[f][c] = alloc2d(B, B); }
    pic_directions2 = (float **)malloc(sizeof(float *) * 2 * B);
    float *d = (float *)calloc(4 * B * B, sizeof(float));
    for (int i = 0; i < 2 * B; i++) pic_directions2[i] = d + i * 2 * B;
    inited = 1;
  }
  for (int f = 0; f < HN - 1; f++)
    for (int y = 0; y < B; y++)
      for (int x = 0; x < B; x++) {
        refPicsData[f][comp][y][x] = org_hist[f * B * B + y * B + x];
        srcPicsData[f][comp][y][x] = rec_hist[f * B * B + y * B + x];
      }
  for (int i = 0; i < 4 * B * B; i++) pic_directions2[0][i] = dirs[i];
  imgpel **o = alloc2d(B, B), **r = alloc2d(B, B);
  for (int y = 0; y < B; y++)
    for (int x = 0; x < B; x++) {
      o[y][x] = org_hist[(HN - 1) * B * B + y * B + x];
      r[y][x] = rec_hist[(HN - 1) * B * B + y * B + x];
    }
  float v = compute_stVSSIM(o, r, 0, 0, 0, 0, h, w, wint, gama, comp, ssim, ssim3d, stvssim);
  free(o[0]); free(o); free(r[0]); free(r);
  return v;
}

double stv_lambda_2(int qp) { return lambda_2(qp); }
double stv_adjust_lambda(double lambda, double eta) { return adjust_lambda(lambda, eta); }

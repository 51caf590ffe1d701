// cu_timer.cpp -- MEASUREMENT HARNESS (the bench's CPU reference baseline; never shipped).
//
// Linked into a copy of the reference TAppEncoder (oracle/Makefile target _ref/TAppEncoder_cutime)
// with -Wl,--wrap=<TEncCu::compressCtu>: the reference code runs unmodified, and every
// compressCtu call (TEncSlice.cpp:814 -> TEncCu.cpp:228) is timed with the monotonic clock.  At
// exit the per-picture totals go to stderr, one line per POC:
//   cu_time poc <POC> type <slice type> qp <slice QP> nref <L0 refs> ctus <n> seconds <sum>
// so the bench can price exactly the pictures that match its GPU workload (bench.py
// hm_cpu_reference).
#include <sstream>
#include <iostream>
#include <vector>
#include <list>
#include <map>
#include <string>
#include <cstdio>
#include <ctime>
#include "TLibCommon/CommonDef.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComSlice.h"
#include "TLibEncoder/TEncCu.h"

#define CU_SYM _ZN6TEncCu11compressCtuEP10TComDataCU
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

extern "C" void CAT(__real_, CU_SYM)(TEncCu *, TComDataCU *);

namespace {
struct Pic { int type = 0, qp = 0, nref = 0, ctus = 0; double sec = 0; };
struct Times {
  std::map<int, Pic> pics;
  ~Times() {
    for (auto &kv : pics)
      fprintf(stderr, "cu_time poc %d type %d qp %d nref %d ctus %d seconds %.6f\n", kv.first, kv.second.type, kv.second.qp,
              kv.second.nref, kv.second.ctus, kv.second.sec);
  }
};
Times g;
double now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
}  // namespace

extern "C" void CAT(__wrap_, CU_SYM)(TEncCu *self, TComDataCU *ctu) {
  TComSlice *s = ctu->getSlice();
  Pic &p = g.pics[s->getPOC()];
  p.type = s->getSliceType();
  p.qp = s->getSliceQp();
  p.nref = s->getSliceType() == I_SLICE ? 0 : s->getNumRefIdx(REF_PIC_LIST_0);
  const double t0 = now();
  CAT(__real_, CU_SYM)(self, ctu);
  p.sec += now() - t0;
  p.ctus++;
}

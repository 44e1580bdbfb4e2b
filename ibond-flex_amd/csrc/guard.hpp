// Address guards of the test build (round 5; VERDICT r4 "next" item 1).
//
// In libflexpai_xcheck.so (FLEXPAI_XCHECK = 1) the table samplers and their neighbours -- k_fb_digits, k_fbs_fill,
// k_fbs, k_sgp, k_fbp_fin -- check every index they form from data (a digit, a row number) or from the element count
// (digit, pair-tile, output and ciphertext offsets) against the size of the buffer it addresses, as the host
// allocated it (GuardArgs, filled in flexpai.hip). A violation is counted in a device record, the first one is kept
// (site, value, limit, element), and the index is CLAMPED to 0, so the kernel never touches memory outside its
// buffers: a guard trip is a failed call (pai_last_error names the site), never a GPU fault. The product build
// (FLEXPAI_XCHECK = 0) compiles the checks out; its kernels are unchanged.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef FLEXPAI_XCHECK
#define FLEXPAI_XCHECK 0
#endif

namespace fpai {

struct GuardRec {
  unsigned int hits;        // violations counted
  unsigned int site;        // the first violation: GuardSite
  unsigned long long val;   //   the index formed
  unsigned long long lim;   //   the size it had to stay below
  long long elem;           //   the element (or table entry) being processed
};

// Sizes are in the unit the kernel indexes in: rows (table rows per half), words (digits, pairs, outputs).
struct GuardArgs {
  GuardRec* rec;              // null: no checks (the product build never sets it)
  unsigned long long rows;    // table rows per half (K 2^W)
  unsigned long long digits;  // digit words ([halves][K][n])
  unsigned long long out;     // output words (pair tiles, pair rows, or ciphertext words)
  unsigned long long in;      // input words (k_fbp_fin: the pair tiles it reads)
};

enum GuardSite : unsigned int {
  GS_NONE = 0,
  GS_DIG_OUT = 1,      // k_fb_digits: digit store
  GS_FILL_LOHI = 2,    // k_fbs_fill: lo/hi entry and inverse reads
  GS_FILL_ROW = 3,     // k_fbs_fill: row store
  GS_FBS_DIGIT = 4,    // k_fbs: digit load offset
  GS_FBS_DVAL = 5,     // k_fbs: digit value < 2^W
  GS_FBS_ROW = 6,      // k_fbs: row index < K 2^W (row DMA and b R loads)
  GS_FBS_OUT = 7,      // k_fbs: pair tile store
  GS_SGP_DIGIT = 8,    // k_sgp: digit load offset
  GS_SGP_DVAL = 9,     // k_sgp: digit value < 2^W
  GS_SGP_ROW = 10,     // k_sgp: row index (a-half DMA and b loads)
  GS_SGP_OUT = 11,     // k_sgp: pair row store
  GS_FIN_TILE = 12,    // k_fbp_fin: pair tile reads (DMA and direct)
  GS_FIN_CT = 13,      // k_fbp_fin: ciphertext store
};

inline const char* guard_site_name(unsigned int s) {
  static const char* const names[] = {"none",         "k_fb_digits digit store", "k_fbs_fill lo/hi read", "k_fbs_fill row store",
                                      "k_fbs digit load", "k_fbs digit value",     "k_fbs row index",      "k_fbs pair store",
                                      "k_sgp digit load", "k_sgp digit value",     "k_sgp row index",      "k_sgp pair store",
                                      "k_fbp_fin tile read", "k_fbp_fin ciphertext store"};
  return s < sizeof(names) / sizeof(names[0]) ? names[s] : "?";
}

#if FLEXPAI_XCHECK
// v < lim; otherwise the violation is recorded
__device__ __forceinline__ bool guard_ok(const GuardArgs& g, unsigned int site, unsigned long long v, unsigned long long lim,
                                         long long elem) {
  if (g.rec && !(v < lim)) {
    if (atomicAdd(&g.rec->hits, 1u) == 0u) {
      g.rec->site = site;
      g.rec->val = v;
      g.rec->lim = lim;
      g.rec->elem = elem;
    }
    return false;
  }
  return true;
}
// v if v < lim; otherwise the violation is recorded and 0 returned
__device__ __forceinline__ unsigned long long guard_idx(const GuardArgs& g, unsigned int site, unsigned long long v,
                                                        unsigned long long lim, long long elem) {
  return guard_ok(g, site, v, lim, elem) ? v : 0ull;
}
#define FPAI_GUARD_OK(g, site, v, lim, e) ::fpai::guard_ok((g), (site), (v), (lim), (e))
#define FPAI_GUARD_IDX(g, site, v, lim, e) ::fpai::guard_idx((g), (site), (v), (lim), (e))
#else
// the product build: no check, and the arguments are not evaluated (a reference to a kernel argument's member would
// move the whole argument struct to the stack: measured, k_fbs<37> spilled 500 B)
#define FPAI_GUARD_OK(g, site, v, lim, e) true
#define FPAI_GUARD_IDX(g, site, v, lim, e) (v)
#endif

}  // namespace fpai

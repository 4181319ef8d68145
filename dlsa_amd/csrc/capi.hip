// extern "C" entry points of libdlsa_hip.so (declared in include/dlsa_hip.h)
// and the host side of the batched Newton/IRLS driver.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "dlsa_internal.hpp"

namespace dlsa {

static thread_local std::string g_last_error;
static thread_local dlsa_fit_stats g_stats;

void set_error(const std::string& msg) { g_last_error = msg; }

hipError_t ensure_max_lds(const void* kernel, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> done;  // (kernel, device) -> bytes set
  std::lock_guard<std::mutex> lock(mu);
  auto it = done.find({kernel, dev});
  if (it != done.end() && it->second >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done[{kernel, dev}] = bytes;
  return e;
}

#define DLSA_HIP_TRY(expr)                                                            \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                   \
      return DLSA_E_HIP;                                                              \
    }                                                                                 \
  } while (0)

static inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// Chunking: each wave streams a run of consecutive rows of one partition.
// Enough chunks to give every CU several waves, few enough that the partial
// tiles (T*2 KiB per chunk) stay ~1-2% of the X traffic.
struct Plan {
  int P = 0, NT = 0, T = 0, PP = 0;
  int n_chunks = 0;
  int max_chunk_rows = 0;
  std::vector<int64_t> chunk_row0;
  std::vector<int32_t> chunk_rows, chunk_part, part_chunk_begin;
};

// Chunking: ~8192 chunks of consecutive rows of one partition.  The
// cooperative pass runs one 4-wave workgroup per chunk (2 per CU: 512 in
// flight), the per-wave fp64 pass one wave per chunk (4 per CU: 1024 in
// flight), so a launch is whole rounds of either; the partial tiles
// (T * 2 KiB per chunk) stay ~1 % of the X traffic.  Measured at config 2
// (cooperative bf16 / fp64 pass ms): 1024 chunks 22.0 / 42.5, 2048 19.4 /
// 36.6, 4096 18.2 / 34.7, 8192 17.4 / 33.2, 16384 17.0 / 32.8 (but the Newton
// solve reads every chunk's partial tiles: 0.65 -> 0.74 ms per iteration).
// Round 2 (current kernels): ~6144 chunks of at least 4096 rows.  Config 2
// at 16384 rows per chunk (6144 chunks) against the old 8448: 82.8-84.1 vs
// 84.6-91.0 ms alternated on one box, 86.2-86.6 vs 86.3-86.6 on another
// (profiles/r02ap_c2_chunk_ab.txt, r02ar_c2_chunk_ab.txt); at the
// strong-scaling share of config 2 (n = 1.25e7 per GPU, 1525 rows per chunk
// by the old rule) 3072 / 6144-row chunks fit 12.8 / 12.7 ms against 13.5 ms
// (fewer per-chunk prologues and partial tiles; r02am).  Round 5 (current
// kernels, r05j, alternated): at that share 4096 / 6144 / 8192 / 12288 rows
// per chunk fit 11.10-11.28 / 10.70-10.73 / 10.85-10.97 / 10.71-10.81 ms, so the
// floor is 6144 rows (2048 chunks there; config 2 itself is unchanged).
static int auto_rows_per_chunk(int64_t n_total) {
  if (const char* e = env_knob("DLSA_ROWS_PER_CHUNK")) return std::max(64, atoi(e));
  // rounded up to a multiple of 1024: equal partitions then split into whole
  // chunks (config 2: 16384 rows, 6 per partition) instead of a ragged extra one
  int64_t r = (n_total / 6144 + 1023) / 1024 * 1024;
  r = std::max<int64_t>(6144, std::min<int64_t>(r, 131072));
  return (int)r;
}

// rows_used(k) = clamp(ceil(frac * n_k), min_rows, n_k): a prefix of each
// partition (frac = 1: all rows).
static int64_t rows_used(int64_t nk, double frac, int64_t min_rows) {
  if (frac >= 1.0) return nk;
  return std::min(nk, std::max(min_rows, (int64_t)std::ceil(frac * (double)nk)));
}
// the next iteration's approximate pass enqueued before the host reads the
// counters (1) or after (0, A/B; fit_impl's spec_pass)
#ifndef DLSA_SPEC_PASS
#define DLSA_SPEC_PASS 1
#endif
// warm-start row-prefix fractions (ascending, each < 1); DLSA_LEVELS="a,b,..."
// overrides (schedule sweeps, tools/level_sweep.sh), DLSA_LEVELS="" disables.
// A level using more than half of all rows is skipped, so "x,0.5" runs as
// "x" alone at config 2 (odd n_k round up).  Fused pass (config 2,
// profiles/r01m_level_sweep.jsonl, 6-step means): one 1/16 level at a
// 0.2-relative step 101 ms per fit vs 110 ms for 1/16, 1/4 at 0.1 (6 bf16 +
// 1 fp64 launches instead of 9 + 1: the 1/4 level's passes cost more than
// the one full pass they save).  Wide path: 1/16, 1/4 at 0.1, with a level
// dropped when the next has under twice its rows (wide_level_plans; config 5
// runs 1/4 alone) -- other schedules were within noise, slower (1/4 at a
// 0.15 tolerance: 56.4 ms fit, r06h) or triggered a second fp64 Gram pass.
static std::vector<double> warm_level_fracs(bool fused) {
  std::vector<double> f = fused ? std::vector<double>{1.0 / 16.0}
                                : std::vector<double>{1.0 / 16.0, 1.0 / 4.0};
  if (const char* e = env_knob("DLSA_LEVELS")) {
    f.clear();
    for (const char* s = e; *s;) {
      char* end = nullptr;
      const double v = strtod(s, &end);
      if (end == s) break;
      if (v > 0.0 && v < 1.0) f.push_back(v);
      s = (*end == ',') ? end + 1 : end;
    }
  }
  return f;
}
// iteration budget of one warm-start level: at most kLevelIters and at most
// half of what is left of max_iter, so the levels and the full-data level
// together run at most max_iter iterations (sklearn's n_iter_ <= max_iter)
// and the full-data level always gets at least one; max_iter = 1 runs no
// level at all.
constexpr int kLevelIters = 10;
static int iter_budget(bool final_level, int it, int max_iter) {
  if (final_level) return std::max(1, max_iter - it);
  return std::min(kLevelIters, (max_iter - it) / 2);
}
// Pinned host staging of the per-iteration readbacks (running counters +
// phases), grown on demand and kept for the thread's lifetime: a
// hipHostMalloc / hipHostFree pair per fit costs a pinning call (and the free
// an implicit synchronisation) on every call.  Never freed: the process exit
// reclaims it (a thread_local destructor could run after the HIP runtime's).
static int32_t* pinned_staging(size_t n_i32) {
  thread_local int32_t* buf = nullptr;
  thread_local size_t cap = 0;
  if (cap < n_i32) {
    int32_t* nb = nullptr;
    if (hipHostMalloc((void**)&nb, n_i32 * 4, hipHostMallocDefault) != hipSuccess) return nullptr;
    if (buf) (void)hipHostFree(buf);
    buf = nb;
    cap = n_i32;
  }
  return buf;
}

// Pinned host staging of the chunk tables a fit uploads at its start and at
// every warm-start level change.  From pageable vectors hipMemcpyAsync copies
// through the runtime's own staging and returns when the copy is done: the
// first such copy of a process took 16.7 ms at config 2's level change
// (profiles/r06d_first_fit_trace.txt), with the GPU idle behind it.  From
// here the copies are asynchronous.  Thread-local, grown on demand at a fit's
// start (reserve: every plan of the fit), never shrunk; an event after the
// last staged copy guards the reuse by the next fit (a fit that fails early
// returns without its final synchronisation).
struct PinnedArena {
  char* buf = nullptr;
  size_t cap = 0, used = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
};
static PinnedArena& pinned_arena() {
  thread_local PinnedArena a;
  return a;
}
static hipError_t pinned_arena_reserve(size_t bytes) {
  PinnedArena& a = pinned_arena();
  if (a.pending) {
    hipError_t e = hipEventSynchronize(a.done);
    if (e != hipSuccess) return e;
    a.pending = false;
  }
  a.used = 0;
  if (!a.done) {
    hipError_t e = hipEventCreateWithFlags(&a.done, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  if (a.cap >= bytes) return hipSuccess;
  char* nb = nullptr;
  hipError_t e = hipHostMalloc((void**)&nb, bytes, hipHostMallocDefault);
  if (e != hipSuccess) return e;
  if (a.buf) (void)hipHostFree(a.buf);
  a.buf = nb;
  a.cap = bytes;
  return hipSuccess;
}
// bytes one call of staged_upload takes from the arena
static size_t staged_bytes(size_t bytes) { return (size_t)align_up((int64_t)bytes, 64); }
// H2D copy of host data through the arena (pageable copy if it is full)
static hipError_t staged_upload(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  PinnedArena& a = pinned_arena();
  if (!a.buf || a.used + staged_bytes(bytes) > a.cap)
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
  char* p = a.buf + a.used;
  a.used += staged_bytes(bytes);
  memcpy(p, src, bytes);
  hipError_t e = hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipEventRecord(a.done, s);
  if (e == hipSuccess) a.pending = true;
  return e;
}
// arena bytes of one plan's chunk tables (row0, rows, part, partition chunk begins)
static size_t plan_staged_bytes(const Plan& q, int K) {
  return staged_bytes(8 * (size_t)q.n_chunks) + 2 * staged_bytes(4 * (size_t)q.n_chunks) +
         staged_bytes(4 * ((size_t)K + 1));
}
static hipError_t upload_plan_tables(const Plan& q, int K, void* d_row0, void* d_rows,
                                     void* d_part, void* d_pcb, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (q.n_chunks > 0) {
    e = staged_upload(d_row0, q.chunk_row0.data(), 8LL * q.n_chunks, s);
    if (e == hipSuccess) e = staged_upload(d_rows, q.chunk_rows.data(), 4LL * q.n_chunks, s);
    if (e == hipSuccess) e = staged_upload(d_part, q.chunk_part.data(), 4LL * q.n_chunks, s);
  }
  if (e == hipSuccess) e = staged_upload(d_pcb, q.part_chunk_begin.data(), 4LL * (K + 1), s);
  return e;
}

// fewest rows of a warm-start level per parameter (DLSA_LEVEL_ROWS_PER_P
// overrides in knob builds, schedule sweeps)
static int64_t level_rows_per_param() {
  if (const char* e = env_knob("DLSA_LEVEL_ROWS_PER_P")) return std::max<int64_t>(1, atoll(e));
  return 64;
}

// a level stops once its max relative step is below this; DLSA_LEVEL_TOL overrides
static double warm_level_tol(bool fused) {
  if (const char* e = env_knob("DLSA_LEVEL_TOL")) return atof(e);
  return fused ? 0.2 : 0.1;
}

static int64_t level_rows(const int64_t* offsets, int K, double frac, int64_t min_rows) {
  int64_t n = 0;
  for (int k = 0; k < K; ++k) n += std::max<int64_t>(0, rows_used(offsets[k + 1] - offsets[k], frac, min_rows));
  return n;
}

static bool make_plan(const int64_t* offsets, int K, int p, int intercept, int rows_per_chunk,
                      Plan& pl, double frac = 1.0, int64_t min_rows = 0) {
  pl.P = p + (intercept ? 1 : 0);
  pl.NT = (pl.P + 15) / 16;
  pl.T = pl.NT * (pl.NT + 1) / 2;
  pl.PP = 16 * pl.NT;
  // fused pass: chunk size from all rows (a warm-start level keeps the full
  // pass's chunk size: fewer, equally long chunks -- measured as fast)
  const int64_t n_total = offsets[K];
  const int rpc = rows_per_chunk > 0 ? rows_per_chunk : auto_rows_per_chunk(n_total);
  pl.part_chunk_begin.assign(K + 1, 0);
  pl.chunk_row0.clear();
  pl.chunk_rows.clear();
  pl.chunk_part.clear();
  for (int k = 0; k < K; ++k) {
    pl.part_chunk_begin[k] = (int32_t)pl.chunk_row0.size();
    const int64_t a = offsets[k];
    const int64_t nk = offsets[k + 1] - a;
    const int64_t n = rows_used(nk, frac, min_rows);
    if (n <= 0) continue;
    const int64_t nc = (n + rpc - 1) / rpc;
    for (int64_t c = 0; c < nc; ++c) {
      const int64_t r0 = a + n * c / nc, r1 = a + n * (c + 1) / nc;
      pl.chunk_row0.push_back(r0);
      pl.chunk_rows.push_back((int32_t)(r1 - r0));
      pl.chunk_part.push_back(k);
    }
  }
  pl.part_chunk_begin[K] = (int32_t)pl.chunk_row0.size();
  pl.n_chunks = (int)pl.chunk_row0.size();
  pl.max_chunk_rows = 0;
  for (int32_t r : pl.chunk_rows) pl.max_chunk_rows = std::max<int>(pl.max_chunk_rows, r);
  return true;
}

struct Layout {
  int64_t off_row0, off_rows, off_part, off_pcb, off_offsets;
  int64_t off_slabH, off_slabg, off_slabll;
  int64_t off_phase, off_bt, off_llprev, off_thprev, off_dprev, off_counters;
  int64_t off_dmprev, off_stall;
  int64_t off_colmax, off_zcolmax, off_threc;  // Ozaki digit scales (PassArgs)
  int64_t total;
};

static Layout make_layout(const Plan& pl, int K) {
  Layout L;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    int64_t r = o;
    o = align_up(o + bytes, 256);
    return r;
  };
  L.off_row0 = take(8LL * std::max(pl.n_chunks, 1));
  L.off_rows = take(4LL * std::max(pl.n_chunks, 1));
  L.off_part = take(4LL * std::max(pl.n_chunks, 1));
  L.off_pcb = take(4LL * (K + 1));
  L.off_offsets = take(8LL * (K + 1));
  L.off_slabH = take(8LL * std::max(pl.n_chunks, 1) * pl.T * 256);
  L.off_slabg = take(8LL * std::max(pl.n_chunks, 1) * pl.PP);
  L.off_slabll = take(8LL * std::max(pl.n_chunks, 1));
  // the counters and the phases are adjacent (counters first, as in the
  // pinned staging): one readback per iteration
  L.off_counters = take(16 + 4LL * K);
  L.off_phase = L.off_counters + 16;
  L.off_bt = take(4LL * K);
  L.off_llprev = take(8LL * K);
  L.off_thprev = take(8LL * K * pl.P);
  L.off_dprev = take(8LL * K * pl.P);
  L.off_dmprev = take(8LL * K);
  L.off_stall = take(4LL * K);
  L.off_colmax = take(4LL * std::max(pl.n_chunks, 1) * pl.PP);
  L.off_zcolmax = take(4LL * std::max(pl.n_chunks, 1) * pl.PP);
  L.off_threc = take(8LL * K * pl.P);
  L.total = o;
  return L;
}

// ---- wide-P path (P > DLSA_MAX_P_FUSED): row chunks + Gram row groups ------
struct WidePlans {
  Plan rows, gram;
};

// Row pass (exact partitions): ~2048 chunks (one 256-thread workgroup each,
// HBM-bound).  Gram row groups (fused bf16 pass and fp64 Gram pass): >= 256,
// a multiple of 8 so the XCD-aware mappings fill every XCD.
static void make_wide_plans(const int64_t* offsets, int K, int p, int intercept,
                            int rows_per_chunk, WidePlans& wp, double frac = 1.0,
                            int64_t min_rows = 0) {
  // wide path: row-group sizes from the rows this level streams, so a
  // warm-start level fills the chip like a full pass
  const int64_t n_total = level_rows(offsets, K, frac, min_rows);
  const int P = p + (intercept ? 1 : 0);
  const int NB = (P + kWideTile - 1) / kWideTile;
  const int TB = NB * (NB + 1) / 2;
  int rpc_row = (int)std::max<int64_t>(256, std::min<int64_t>(n_total / 2048, 16384));
  // >= 256 row groups: the fused pass runs 2 workgroups per row group above
  // PP = 256 (512 in all, 1 per CU), the fp64 Gram pass TB per row group;
  // measured at config 5 (p = 500), fp64 pass: 64 / 128 / 256 row groups ->
  // 43.8 / 36.8 / 36.1 ms
  const int64_t groups = (std::max<int64_t>(256, (1024 + TB - 1) / TB) + 7) / 8 * 8;
  int rpc_gram = (int)std::max<int64_t>(1024, std::min<int64_t>((n_total + groups - 1) / groups,
                                                                int64_t(1) << 24));
  if (rows_per_chunk > 0) rpc_row = rpc_gram = rows_per_chunk;
  if (const char* e = env_knob("DLSA_WIDE_GRAM_ROWS")) rpc_gram = std::max(64, atoi(e));
  // the Gram kernels address a row group's X with 32-bit buffer offsets
  rpc_gram = (int)std::min<int64_t>(rpc_gram, (int64_t(1) << 30) / (8LL * std::max(p, 1)));
  make_plan(offsets, K, p, intercept, rpc_row, wp.rows, frac, min_rows);
  make_plan(offsets, K, p, intercept, rpc_gram, wp.gram, frac, min_rows);
}

struct WideLayout {
  int64_t off_r_row0, off_r_rows, off_r_part, off_rcb;
  int64_t off_g_row0, off_g_rows, off_g_part, off_gcb;
  int64_t off_offsets, off_w, off_slabg, off_slabll, off_slabG, off_slabgz, off_slabllz, off_H;
  int64_t off_phase, off_bt, off_llprev, off_thprev, off_dprev, off_counters;
  int64_t off_dmprev, off_stall;
  int64_t off_zmax, off_ozE;  // int8 exact Gram: row-chunk max |z|, digit exponents
  // int8 exact Gram digit records (wide_oz.hip): the last region, so that
  // base_total bytes hold everything else; digit_bytes = 0 when the final
  // plan's row groups are too long (> kWideOzMaxRows) or the records would
  // exceed kWideOzMaxDigitBytes (the fp64 Gram runs then)
  int64_t off_digits, digit_bytes, base_total;
  int64_t total;
  int64_t cap_rows, cap_gram;  // row-chunk / Gram-row-group capacity of the tables and slabs
};

// Largest digit-record region a wide fit asks for (above it: fp64 Gram).
constexpr int64_t kWideOzMaxDigitBytes = int64_t(32) << 30;

// Sized for the largest chunk counts over ALL level plans: a warm-start
// level's row groups are sized from its own (smaller) row count, so with
// uneven partitions it can have more row chunks / Gram row groups than the
// final plan (e.g. P = 512, n_k = [1e7, 1e5, 1e5]: 258 vs 257 Gram groups).
static WideLayout make_wide_layout(const std::vector<WidePlans>& plans, int K, int64_t n_total,
                                   int P) {
  const int NB = (P + kWideTile - 1) / kWideTile;
  const int64_t PP = (int64_t)kWideTile * NB;
  const int64_t TB = NB * (NB + 1) / 2;
  int64_t nr = 1, ng = 1;
  for (const WidePlans& wp : plans) {
    nr = std::max<int64_t>(nr, wp.rows.n_chunks);
    ng = std::max<int64_t>(ng, wp.gram.n_chunks);
  }
  WideLayout L;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    int64_t r = o;
    o = align_up(o + bytes, 256);
    return r;
  };
  L.off_r_row0 = take(8 * nr);
  L.off_r_rows = take(4 * nr);
  L.off_r_part = take(4 * nr);
  L.off_rcb = take(4LL * (K + 1));
  L.off_g_row0 = take(8 * ng);
  L.off_g_rows = take(4 * ng);
  L.off_g_part = take(4 * ng);
  L.off_gcb = take(4LL * (K + 1));
  L.off_offsets = take(8LL * (K + 1));
  L.off_w = take(8 * std::max<int64_t>(n_total, 1));
  L.off_slabg = take(8 * nr * PP);
  L.off_slabll = take(8 * nr);
  L.off_slabG = take(8 * ng * TB * kWideTile * kWideTile);
  L.off_slabgz = take(8 * ng * PP);
  L.off_slabllz = take(8 * ng);
  L.off_H = take(8LL * K * PP * PP);
  // the counters and the phases are adjacent (counters first, as in the
  // pinned staging): one readback per iteration
  L.off_counters = take(16 + 4LL * K);
  L.off_phase = L.off_counters + 16;
  L.off_bt = take(4LL * K);
  L.off_llprev = take(8LL * K);
  L.off_thprev = take(8LL * K * P);
  L.off_dprev = take(8LL * K * P);
  L.off_dmprev = take(8LL * K);
  L.off_stall = take(4LL * K);
  L.off_zmax = take(4 * nr * PP);
  L.off_ozE = take(4 * ng * PP);
  L.base_total = o;
  const Plan& fg = plans.back().gram;
  int max_grows = 0;
  for (int c = 0; c < fg.n_chunks; ++c) max_grows = std::max(max_grows, fg.chunk_rows[c]);
  const int64_t db = wide_oz_digit_bytes(fg.n_chunks, max_grows, (int)PP);
  L.digit_bytes = (max_grows <= kWideOzMaxRows && db <= kWideOzMaxDigitBytes) ? db : 0;
  L.off_digits = take(L.digit_bytes);
  L.total = o;
  L.cap_rows = nr;
  L.cap_gram = ng;
  return L;
}

// The wide path's plans: the warm-start levels (logistic, warm_start) then
// all rows.  A level that would stream more than half of the rows is
// skipped (it would cost more than the full passes it saves).  A level
// whose row count is less than twice the previous level's replaces it: the
// min_rows floor can lift a small fraction to nearly the next one (config 5:
// 1/16 of n_k = 156250 is raised to 64 x 500 = 32000 rows, the 1/4 level has
// 39063), and two levels that close cost a level's iterations twice for the
// same start.  Config 5, one box, 4 A/B pairs (profiles/r06h_level_ab.txt):
// 1/16 + 1/4 10 iterations, fit 54.1-54.2 ms; 1/4 alone 9, 52.7-52.8 ms.
static std::vector<WidePlans> wide_level_plans(const int64_t* offsets, int K, int p, int intercept,
                                               int rows_per_chunk, bool levels) {
  std::vector<WidePlans> plans;
  const int P = p + (intercept ? 1 : 0);
  if (levels) {
    const int64_t min_rows = std::max<int64_t>(2048, level_rows_per_param() * P);
    int64_t prev_rows = 0;
    for (double frac : warm_level_fracs(false)) {
      WidePlans q;
      make_wide_plans(offsets, K, p, intercept, rows_per_chunk, q, frac, min_rows);
      int64_t rows = 0;
      for (int c = 0; c < q.rows.n_chunks; ++c) rows += q.rows.chunk_rows[c];
      if (rows > offsets[K] / 2 || q.rows.n_chunks == 0) continue;
      if (!plans.empty() && rows < 2 * prev_rows) plans.pop_back();
      plans.push_back(std::move(q));
      prev_rows = rows;
    }
  }
  WidePlans fin;
  make_wide_plans(offsets, K, p, intercept, rows_per_chunk, fin);
  plans.push_back(std::move(fin));
  return plans;
}

static int check_offsets(const int64_t* offsets, int K) {
  if (!offsets || K < 1) {
    set_error("offsets must be a host array of K+1 >= 2 entries");
    return DLSA_E_INVALID;
  }
  if (offsets[0] != 0) {
    set_error("offsets[0] must be 0");
    return DLSA_E_INVALID;
  }
  for (int k = 0; k < K; ++k)
    if (offsets[k + 1] < offsets[k]) {
      set_error("offsets must be non-decreasing");
      return DLSA_E_INVALID;
    }
  for (int k = 0; k < K; ++k)
    if (offsets[k + 1] - offsets[k] > (int64_t)INT32_MAX) {
      set_error("a partition holds more than 2^31-1 rows");
      return DLSA_E_INVALID;
    }
  return DLSA_OK;
}

}  // namespace dlsa

using namespace dlsa;

extern "C" {

void dlsa_fit_options_default(dlsa_fit_options* opt) {
  if (!opt) return;
  memset(opt, 0, sizeof(*opt));
  opt->hessian_mode = DLSA_HESSIAN_MIXED;
  opt->switch_tol = 1e-6;
  opt->warm_start = 1;
}

const char* dlsa_last_error(void) { return g_last_error.c_str(); }

const char* dlsa_build_info(void) {
  return "libdlsa_hip gfx950 (CDNA4): fused IRLS passes over an LDS-DMA ring (bf16 16x16x32 "
         "approximate Hessians; exact Hessians as int8 16x16x64 digit-slice sums or f64 "
         "16x16x4 MFMA), wide 128x128 Gram tiles, LDS Cholesky Newton update, host LARS";
}

int64_t dlsa_logistic_workspace_bytes(const int64_t* offsets, int32_t K, int32_t p,
                                      int32_t fit_intercept, int32_t rows_per_chunk) {
  if (check_offsets(offsets, K) != DLSA_OK) return -1;
  const int P = p + (fit_intercept ? 1 : 0);
  if (P > DLSA_MAX_P_FUSED)  // sized for the warm-start levels too (an upper bound)
    return make_wide_layout(wide_level_plans(offsets, K, p, fit_intercept, rows_per_chunk, true),
                            K, offsets[K], P)
        .total;
  Plan pl;
  make_plan(offsets, K, p, fit_intercept, rows_per_chunk, pl);
  return make_layout(pl, K).total;
}

int dlsa_last_fit_stats(dlsa_fit_stats* out) {
  if (!out) return DLSA_E_INVALID;
  *out = g_stats;
  return DLSA_OK;
}

}  // extern "C"

namespace dlsa {

// Rows a pass of phase `ph` streams: the rows (in this level's plan) of the
// partitions whose phase is ph.  The partition phases are read back with the
// per-iteration counters (stats only: rows_fp32 / rows_fp64).
static std::vector<int64_t> plan_part_rows(const Plan& q, int K) {
  std::vector<int64_t> r(K, 0);
  for (int k = 0; k < K; ++k)
    for (int c = q.part_chunk_begin[k]; c < q.part_chunk_begin[k + 1]; ++c) r[k] += q.chunk_rows[c];
  return r;
}
static int64_t phase_rows(const std::vector<int64_t>& part_rows, const int32_t* phase,
                          int ph) {
  int64_t n = 0;
  for (size_t k = 0; k < part_rows.size(); ++k)
    if (phase[k] == ph) n += part_rows[k];
  return n;
}

// DLSA_TRACE=1: per-iteration max |step| over all partitions (diagnostics;
// copies theta and the last step to the host, so only for investigation)
static int running_total(const int* n_running) {
  int n = 0;
  for (int ph = 0; ph < kRunPhases; ++ph) n += n_running[ph];
  return n;
}

static hipError_t trace_iteration(int K, int P, const double* theta, const double* dprev,
                                  size_t lvl, int it, const int* n_running) {
  std::vector<double> th((size_t)K * P), dp((size_t)K * P);
  hipError_t e = hipMemcpy(th.data(), theta, 8LL * K * P, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(dp.data(), dprev, 8LL * K * P, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  double dmax = 0.0, tmax = 0.0;
  for (size_t i = 0; i < th.size(); ++i) {
    dmax = std::max(dmax, std::fabs(dp[i]));
    tmax = std::max(tmax, std::fabs(th[i]));
  }
  fprintf(stderr,
          "[dlsa trace] level %zu iter %d: max|step| %.3e max|theta| %.3e running approx %d "
          "f32x %d f64 %d\n",
          lvl, it, dmax, tmax, n_running[PHASE_F32], n_running[PHASE_F32X], n_running[PHASE_F64]);
  return hipSuccess;
}

// Event timer of the fit's stream (record_timing only).  A pair of events
// brackets every launch; the elapsed times are read after the fit's final
// stream synchronisation (flush), so timing adds no host round trip per
// launch and the launches stay queued back to back.
struct StreamTimer {
  hipStream_t stream;
  bool on;
  std::vector<hipEvent_t> ev;        // 2 per recorded launch, reused across calls
  std::vector<double*> dst_a, dst_b; // accumulators of each recorded launch
  size_t used = 0;
  hipError_t init() { return hipSuccess; }
  ~StreamTimer() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  template <typename F>
  hipError_t operator()(double* acc, F&& launch, double* acc2 = nullptr) {
    if (!on) return launch();
    if (2 * used + 2 > ev.size()) {
      for (int i = 0; i < 2; ++i) {
        hipEvent_t e = nullptr;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return r;
        ev.push_back(e);
      }
    }
    hipError_t e = hipEventRecord(ev[2 * used], stream);
    if (e == hipSuccess) e = launch();
    if (e == hipSuccess) e = hipEventRecord(ev[2 * used + 1], stream);
    if (e != hipSuccess) return e;
    dst_a.push_back(acc);
    dst_b.push_back(acc2);
    ++used;
    return hipSuccess;
  }
  // after the stream has been synchronised
  hipError_t flush() {
    for (size_t i = 0; i < used; ++i) {
      float ms = 0.f;
      hipError_t e = hipEventSynchronize(ev[2 * i + 1]);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
      if (e != hipSuccess) return e;
      *dst_a[i] += ms;
      if (dst_b[i]) *dst_b[i] += ms;
    }
    used = 0;
    dst_a.clear();
    dst_b.clear();
    return hipSuccess;
  }
};

// P > DLSA_MAX_P_FUSED (wide_pass.hip): per Newton iteration the fused bf16
// pass (PHASE_F32 partitions) and/or the row + fp64 Gram passes (PHASE_F64),
// the deterministic partial-tile assembly and the per-partition
// blocked-Cholesky update.  Same warm-start
// levels, phases, state machine and outputs as the fused path.
static int fit_wide(int family, const double* X, const double* y, const int64_t* offsets,
                    int32_t K, int32_t p, int32_t fit_intercept, const double* center,
                    const double* scale, int32_t max_iter, double tol, double* theta,
                    double* sig_inv, double* sig_inv_theta, double* loglik, int32_t* iters,
                    int32_t* status, const dlsa_fit_options& opt, hipStream_t stream,
                    std::chrono::steady_clock::time_point t_start) {
  const int P = p + (fit_intercept ? 1 : 0);
  const int NB = (P + kWideTile - 1) / kWideTile;
  const int64_t n_total = offsets[K];
  const std::vector<WidePlans> plans = wide_level_plans(
      offsets, K, p, fit_intercept, opt.rows_per_chunk,
      family == FAMILY_LOGISTIC && opt.warm_start);
  const WideLayout L = make_wide_layout(plans, K, n_total, P);
  g_stats.n_chunks = plans.back().gram.n_chunks;

  // The exact Gram pass runs on the int8 matrix cores (wide_oz.hip) in mixed
  // mode when the final plan's row groups are <= kWideOzMaxRows rows and its
  // digit records fit the workspace: the caller's (dlsa_logistic_workspace_bytes
  // counts them) or the one allocated here.  Without room for them -- a
  // caller workspace of at least base_total but less than total bytes, a
  // failed allocation, or opt.oz_max_bytes below the records' size -- the
  // fp64 Gram runs (stats.oz_fallbacks).  DLSA_EXACT_FP64: always the fp64 Gram.
  bool use_wide_oz = opt.exact_pass != DLSA_EXACT_FP64 && family == FAMILY_LOGISTIC &&
                     opt.hessian_mode == DLSA_HESSIAN_MIXED && L.digit_bytes > 0;
  if (use_wide_oz && opt.oz_max_bytes > 0 && L.digit_bytes > opt.oz_max_bytes) {
    use_wide_oz = false;
    g_stats.oz_fallbacks++;
  }
  char* ws = (char*)opt.workspace;
  bool owned = false;
  if (!ws) {
    hipError_t e = hipErrorOutOfMemory;
    if (use_wide_oz) {
      e = hipMallocAsync((void**)&ws, L.total, stream);
      if (e != hipSuccess) {
        (void)hipGetLastError();  // out of memory: the fp64 Gram needs no records
        ws = nullptr;
        use_wide_oz = false;
        g_stats.oz_fallbacks++;
      }
    }
    if (!ws) DLSA_HIP_TRY(hipMallocAsync((void**)&ws, L.base_total, stream));
    owned = true;
  } else if (opt.workspace_bytes < L.base_total) {
    set_error("workspace too small: need " + std::to_string(L.total) + " bytes");
    return DLSA_E_WORKSPACE;
  } else if (use_wide_oz && opt.workspace_bytes < L.total) {
    use_wide_oz = false;
    g_stats.oz_fallbacks++;
  }
  struct Free {
    char* p;
    bool own;
    hipStream_t s;
    ~Free() {
      if (own && p) (void)hipFreeAsync(p, s);
    }
  } freer{ws, owned, stream};
  auto at = [&](int64_t off) { return (void*)(ws + off); };
  int64_t* d_offsets = (int64_t*)at(L.off_offsets);
  int32_t* d_rcb = (int32_t*)at(L.off_rcb);
  int32_t* d_gcb = (int32_t*)at(L.off_gcb);
  double* d_H = (double*)at(L.off_H);
  int32_t* d_phase = (int32_t*)at(L.off_phase);
  int32_t* d_bt = (int32_t*)at(L.off_bt);
  double* d_llprev = (double*)at(L.off_llprev);
  int32_t* d_cnt = (int32_t*)at(L.off_counters);

  WideArgs wa;
  memset(&wa, 0, sizeof(wa));
  wa.X = X;
  wa.y = y;
  wa.rc_row0 = (const int64_t*)at(L.off_r_row0);
  wa.rc_rows = (const int32_t*)at(L.off_r_rows);
  wa.rc_part = (const int32_t*)at(L.off_r_part);
  wa.gc_row0 = (const int64_t*)at(L.off_g_row0);
  wa.gc_rows = (const int32_t*)at(L.off_g_rows);
  wa.gc_part = (const int32_t*)at(L.off_g_part);
  wa.phase = d_phase;
  wa.theta = theta;
  wa.center = center;
  wa.scale = scale;
  wa.w = (double*)at(L.off_w);
  wa.slab_g = (double*)at(L.off_slabg);
  wa.slab_ll = (double*)at(L.off_slabll);
  wa.slab_G = (double*)at(L.off_slabG);
  wa.slab_gz = (double*)at(L.off_slabgz);
  wa.slab_llz = (double*)at(L.off_slabllz);
  wa.p = p;
  wa.P = P;
  wa.intercept = fit_intercept ? 1 : 0;
  wa.NB = NB;

  auto upload_plan = [&](const Plan& q, int64_t o_row0, int64_t o_rows, int64_t o_part,
                         int32_t* d_cb) -> hipError_t {
    return upload_plan_tables(q, K, at(o_row0), at(o_rows), at(o_part), d_cb, stream);
  };
  {
    size_t need = staged_bytes(8 * ((size_t)K + 1));
    for (const WidePlans& q : plans) need += plan_staged_bytes(q.rows, K) + plan_staged_bytes(q.gram, K);
    DLSA_HIP_TRY(pinned_arena_reserve(need));
  }
  DLSA_HIP_TRY(staged_upload(d_offsets, offsets, 8LL * (K + 1), stream));

  // MIXED / MIXED_F32: bf16-MFMA Gram passes until the step is below
  // switch_tol, then fp64 Gram passes (the fused path's phase machine)
  const int start_phase =
      (opt.hessian_mode == DLSA_HESSIAN_FP64 || family == FAMILY_GAUSSIAN) ? PHASE_F64 : PHASE_F32;
  DLSA_HIP_TRY(launch_fit_init(d_offsets, K, P, start_phase, theta, d_phase, d_bt, iters, status,
                               d_llprev, sig_inv, loglik, stream));
  int n_running[kRunPhases] = {0, 0, 0};
  for (int k = 0; k < K; ++k)
    if (offsets[k + 1] > offsets[k]) n_running[start_phase]++;

  SolveArgs sa;
  memset(&sa, 0, sizeof(sa));
  sa.theta = theta;
  sa.dm_prev = (double*)at(L.off_dmprev);
  sa.stall = (int32_t*)at(L.off_stall);
  sa.escalate_to = PHASE_F64;  // no fp32 fused wide pass: bf16 -> fp64
  sa.theta_prev = (double*)at(L.off_thprev);
  sa.delta_prev = (double*)at(L.off_dprev);
  sa.ll_prev = d_llprev;
  sa.phase = d_phase;
  sa.backtracks = d_bt;
  sa.iters = iters;
  sa.status = status;
  sa.counters = d_cnt;
  sa.sig_inv = sig_inv;
  sa.loglik = loglik;
  sa.P = P;
  sa.family = family;
  sa.tol = tol;
  sa.switch_tol = opt.switch_tol;

  const bool standardize = center != nullptr;
  StreamTimer timed{stream, opt.record_timing != 0};
  DLSA_HIP_TRY(timed.init());
  int32_t* h_cnt = pinned_staging(4 + (size_t)K);
  if (!h_cnt) {
    set_error("pinned host staging allocation failed");
    return DLSA_E_HIP;
  }
  int32_t* h_phase = h_cnt + 4;  // [K] phases (pinned: no staging copy per iteration)

  // The row pass of an int8 exact Gram also records each row chunk's max
  // |sqrt(w) x|, from which the scale kernel takes the digit exponents of
  // every Gram row group.
  const Plan& fg = plans.back().gram;
  int max_grows = 0;
  for (int c = 0; c < fg.n_chunks; ++c) max_grows = std::max(max_grows, fg.chunk_rows[c]);
  WideOzArgs woz;
  memset(&woz, 0, sizeof(woz));
  woz.rcb = d_rcb;
  woz.zmax = (const uint32_t*)at(L.off_zmax);
  woz.E = (int32_t*)at(L.off_ozE);
  woz.maxblk = (max_grows + 31) / 32;
  woz.D = use_wide_oz ? (int8_t*)at(L.off_digits) : nullptr;
  auto exact_gram = [&](const WidePlans& q, bool final_level) -> hipError_t {
    const bool oz = use_wide_oz && final_level;
    wa.slab_zmax = oz ? (uint32_t*)at(L.off_zmax) : nullptr;
    hipError_t e = timed(&g_stats.ms_wide_row, [&] {
      return launch_wide_row(wa, standardize, family, q.rows.n_chunks, stream);
    });
    wa.slab_zmax = nullptr;
    if (e != hipSuccess) return e;
    if (!oz)
      return timed(
          &g_stats.ms_wide_gram, [&] { return launch_wide_gram(wa, standardize, stream); },
          &g_stats.ms_pass_fp64);
    g_stats.passes_oz++;
    return timed(
        &g_stats.ms_wide_gram,
        [&] {
          hipError_t e2 = launch_wide_oz_scale(wa, woz, stream);
          if (e2 == hipSuccess) e2 = launch_wide_oz_digits(wa, woz, standardize, stream);
          if (e2 == hipSuccess) e2 = launch_wide_oz_gram(wa, woz, stream);
          return e2;
        },
        &g_stats.ms_pass_fp64);
  };

  int it = 0;
  for (size_t lvl = 0; lvl < plans.size(); ++lvl) {
    const WidePlans& q = plans[lvl];
    const bool final_level = lvl + 1 == plans.size();
    if (q.rows.n_chunks > L.cap_rows || q.gram.n_chunks > L.cap_gram) {
      set_error("internal: wide plan exceeds its workspace layout");
      return DLSA_E_INVALID;
    }
    DLSA_HIP_TRY(upload_plan(q.rows, L.off_r_row0, L.off_r_rows, L.off_r_part, d_rcb));
    DLSA_HIP_TRY(upload_plan(q.gram, L.off_g_row0, L.off_g_rows, L.off_g_part, d_gcb));
    wa.n_gchunks = q.gram.n_chunks;
    const std::vector<int64_t> part_rows = plan_part_rows(q.rows, K);
    if (lvl > 0) {
      DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
      DLSA_HIP_TRY(launch_level_reset(K, P, start_phase, d_phase, status, d_llprev, d_bt, theta,
                                      d_cnt, stream));
      DLSA_HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 16 + 4LL * K, hipMemcpyDeviceToHost, stream));
    } else {
      DLSA_HIP_TRY(hipMemcpyAsync(h_phase, d_phase, 4LL * K, hipMemcpyDeviceToHost, stream));
    }
    DLSA_HIP_TRY(hipStreamSynchronize(stream));
    if (lvl > 0)
      for (int ph = 0; ph < kRunPhases; ++ph) n_running[ph] = h_cnt[ph];
    sa.subsample = final_level ? 0 : 1;
    sa.level_tol = warm_level_tol(false);
    sa.switch_tol = final_level ? opt.switch_tol : 0.0;
    const int it_end = it + iter_budget(final_level, it, max_iter);
    if (it_end <= it) continue;  // no budget left for this warm-start level
    DLSA_HIP_TRY(hipMemsetAsync(sa.dm_prev, 0, 8LL * K, stream));
    DLSA_HIP_TRY(hipMemsetAsync(sa.stall, 0, 4LL * K, stream));
    for (; it < it_end && running_total(n_running) > 0 && q.rows.n_chunks > 0; ++it) {
      // approximate partitions: one fused pass (gradient + bf16 Hessian)
      if (n_running[PHASE_F32] > 0) {
        DLSA_HIP_TRY(timed(
            &g_stats.ms_wide_gram, [&] { return launch_wide_fused(wa, standardize, stream); },
            &g_stats.ms_pass_fp32));
        g_stats.passes_fp32++;
        g_stats.rows_fp32 += phase_rows(part_rows, h_phase, PHASE_F32);
      }
      // exact partitions: row pass (gradient, w) + the exact Gram pass
      if (n_running[PHASE_F64] > 0) {
        DLSA_HIP_TRY(exact_gram(q, final_level));
        g_stats.passes_fp64++;
        g_stats.rows_fp64 += phase_rows(part_rows, h_phase, PHASE_F64);
      }
      DLSA_HIP_TRY(timed(&g_stats.ms_wide_assemble,
                         [&] { return launch_wide_assemble(wa, d_gcb, d_H, K, stream); }));
      DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
      DLSA_HIP_TRY(timed(&g_stats.ms_solve,
                         [&] { return launch_wide_newton(sa, wa, d_rcb, d_gcb, d_H, K, stream); }));
      // counters + phases in one copy (adjacent on both sides)
      DLSA_HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 16 + 4LL * K, hipMemcpyDeviceToHost, stream));
      DLSA_HIP_TRY(hipStreamSynchronize(stream));
      for (int ph = 0; ph < kRunPhases; ++ph) n_running[ph] = h_cnt[ph];
      if (getenv("DLSA_TRACE"))
        DLSA_HIP_TRY(trace_iteration(K, P, theta, sa.delta_prev, lvl, it, n_running));
    }
  }
  g_stats.iterations = it;
  // polish: partitions the budget left running get Sig_inv = X^T W X at the
  // theta they return (row pass + fp64 Gram pass, no step)
  if (family == FAMILY_LOGISTIC && running_total(n_running) > 0 && plans.back().rows.n_chunks > 0) {
    const WidePlans& q = plans.back();
    DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
    DLSA_HIP_TRY(launch_polish_mark(K, d_phase, status, d_cnt, stream));
    DLSA_HIP_TRY(hipMemcpyAsync(h_phase, d_phase, 4LL * K, hipMemcpyDeviceToHost, stream));
    DLSA_HIP_TRY(hipStreamSynchronize(stream));
    const std::vector<int64_t> part_rows = plan_part_rows(q.rows, K);
    DLSA_HIP_TRY(exact_gram(q, true));
    g_stats.passes_fp64++;
    g_stats.rows_fp64 += phase_rows(part_rows, h_phase, PHASE_F64);
    g_stats.polish_partitions = running_total(n_running);
    DLSA_HIP_TRY(timed(&g_stats.ms_wide_assemble,
                       [&] { return launch_wide_assemble(wa, d_gcb, d_H, K, stream); }));
    sa.eval_only = 1;
    sa.subsample = 0;
    DLSA_HIP_TRY(timed(&g_stats.ms_solve,
                       [&] { return launch_wide_newton(sa, wa, d_rcb, d_gcb, d_H, K, stream); }));
    sa.eval_only = 0;
  }
  DLSA_HIP_TRY(launch_fit_finalize(K, P, theta, sig_inv, sig_inv_theta, status, stream));
  DLSA_HIP_TRY(hipStreamSynchronize(stream));
  g_stats.ms_total =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start)
          .count();
  DLSA_HIP_TRY(timed.flush());
  return DLSA_OK;
}

static int fit_impl(int family, const double* X, const double* y, const int64_t* offsets,
                    int32_t K, int32_t p, int32_t fit_intercept, const double* center,
                    const double* scale, int32_t max_iter, double tol, double* theta,
                    double* sig_inv, double* sig_inv_theta, double* loglik, int32_t* iters,
                    int32_t* status, const dlsa_fit_options* opt_in, void* stream_) {
  const auto t_start = std::chrono::steady_clock::now();
  g_last_error.clear();
  memset(&g_stats, 0, sizeof(g_stats));
  hipStream_t stream = (hipStream_t)stream_;
  dlsa_fit_options opt;
  if (opt_in)
    opt = *opt_in;
  else
    dlsa_fit_options_default(&opt);
  if (opt.switch_tol <= 0) opt.switch_tol = 1e-6;

  int rc = check_offsets(offsets, K);
  if (rc != DLSA_OK) return rc;
  if (p < 0 || (p == 0 && !fit_intercept)) {
    set_error("p must be >= 1 (or 0 with an intercept)");
    return DLSA_E_INVALID;
  }
  const int P = p + (fit_intercept ? 1 : 0);
  if (P > DLSA_MAX_P) {
    set_error("P = p + intercept > " + std::to_string(DLSA_MAX_P) + " is not supported");
    return DLSA_E_UNSUPPORTED;
  }
  if ((center == nullptr) != (scale == nullptr)) {
    set_error("center and scale must both be given or both be NULL");
    return DLSA_E_INVALID;
  }
  if (!theta || !sig_inv || !sig_inv_theta || !loglik || !iters || !status) {
    set_error("null output pointer");
    return DLSA_E_INVALID;
  }
  const int64_t n_total = offsets[K];
  if (n_total > 0 && (!X || !y)) {
    set_error("null X or y");
    return DLSA_E_INVALID;
  }
  if (max_iter < 1) max_iter = 1;
  if (!(tol > 0)) tol = 1e-10;
  if (family == FAMILY_GAUSSIAN) max_iter = 1;  // closed form: one exact fp64 pass
  if (P > DLSA_MAX_P_FUSED)
    return fit_wide(family, X, y, offsets, K, p, fit_intercept, center, scale, max_iter, tol,
                    theta, sig_inv, sig_inv_theta, loglik, iters, status, opt, stream, t_start);

  Plan pl;
  make_plan(offsets, K, p, fit_intercept, opt.rows_per_chunk, pl);
  const Layout L = make_layout(pl, K);
  g_stats.n_chunks = pl.n_chunks;

  char* ws = (char*)opt.workspace;
  bool owned = false;
  if (!ws) {
    DLSA_HIP_TRY(hipMallocAsync((void**)&ws, L.total, stream));
    owned = true;
  } else if (opt.workspace_bytes < L.total) {
    set_error("workspace too small: need " + std::to_string(L.total) + " bytes");
    return DLSA_E_WORKSPACE;
  }
  struct Free {
    char* p;
    bool own;
    hipStream_t s;
    ~Free() {
      if (own && p) (void)hipFreeAsync(p, s);
    }
  } freer{ws, owned, stream};

  auto at = [&](int64_t off) { return (void*)(ws + off); };
  int64_t* d_row0 = (int64_t*)at(L.off_row0);
  int32_t* d_rows = (int32_t*)at(L.off_rows);
  int32_t* d_part = (int32_t*)at(L.off_part);
  int32_t* d_pcb = (int32_t*)at(L.off_pcb);
  int64_t* d_offsets = (int64_t*)at(L.off_offsets);
  double* slabH = (double*)at(L.off_slabH);
  double* slabg = (double*)at(L.off_slabg);
  double* slabll = (double*)at(L.off_slabll);
  int32_t* d_phase = (int32_t*)at(L.off_phase);
  int32_t* d_bt = (int32_t*)at(L.off_bt);
  double* d_llprev = (double*)at(L.off_llprev);
  double* d_thprev = (double*)at(L.off_thprev);
  double* d_dprev = (double*)at(L.off_dprev);
  int32_t* d_cnt = (int32_t*)at(L.off_counters);

  auto upload = [&](const Plan& q) -> hipError_t {
    return upload_plan_tables(q, K, d_row0, d_rows, d_part, d_pcb, stream);
  };
  // (the arena is reserved below, once the warm-start level plans are known)

  // warm-start levels: Newton on row prefixes (1/16, 1/4) before all rows
  std::vector<Plan> plans;
  if (family == FAMILY_LOGISTIC && opt.warm_start) {
    const int64_t min_rows = std::max<int64_t>(2048, level_rows_per_param() * pl.P);
    for (double frac : warm_level_fracs(true)) {
      Plan q;
      make_plan(offsets, K, p, fit_intercept, opt.rows_per_chunk, q, frac, min_rows);
      int64_t rows = 0;
      for (int c = 0; c < q.n_chunks; ++c) rows += q.chunk_rows[c];
      if (rows <= n_total / 2 && q.n_chunks > 0) plans.push_back(std::move(q));
    }
  }
  plans.push_back(pl);
  {
    size_t need = staged_bytes(8 * ((size_t)K + 1));
    for (const Plan& q : plans) need += plan_staged_bytes(q, K);
    DLSA_HIP_TRY(pinned_arena_reserve(need));
  }
  DLSA_HIP_TRY(staged_upload(d_offsets, offsets, 8LL * (K + 1), stream));

  if (family == FAMILY_GAUSSIAN) max_iter = 1;  // closed form: one exact fp64 pass
  const int start_phase =
      (opt.hessian_mode == DLSA_HESSIAN_FP64 || family == FAMILY_GAUSSIAN) ? PHASE_F64 : PHASE_F32;
  DLSA_HIP_TRY(launch_fit_init(d_offsets, K, P, start_phase, theta, d_phase, d_bt, iters, status,
                               d_llprev, sig_inv, loglik, stream));

  int n_running[kRunPhases] = {0, 0, 0};
  for (int k = 0; k < K; ++k)
    if (offsets[k + 1] > offsets[k]) n_running[start_phase]++;

  PassArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.X = X;
  pa.y = y;
  pa.chunk_row0 = d_row0;
  pa.chunk_rows = d_rows;
  pa.chunk_part = d_part;
  pa.phase = d_phase;
  pa.theta = theta;
  pa.center = center;
  pa.scale = scale;
  pa.slab_H = slabH;
  pa.slab_g = slabg;
  pa.slab_ll = slabll;
  if (n_total > 0) {
    const uintptr_t xend = (uintptr_t)(X + n_total * (int64_t)p);
    pa.x_last16 = ((xend + 15) & ~(uintptr_t)15) - 16;
    pa.y_last4 = (uintptr_t)(y + n_total) - 4;
  }
  pa.p = p;
  pa.P = P;
  pa.intercept = fit_intercept ? 1 : 0;
  pa.waves = opt.exact_waves;
  const int approx_prec = opt.hessian_mode == DLSA_HESSIAN_MIXED_F32 ? PREC_F32 : PREC_BF16;
  // cooperative-pass LDS ring: two workgroups per CU (P <= 112) so that one's
  // row phase and barrier waits overlap the other's tile phase (measured
  // 27.4 -> 21.8 ms per bf16 pass at config 2 against one workgroup with a
  // deeper ring)
  pa.slot_bytes = coop_slot_bytes(pl.NT, p);
  {
    const int wg_per_cu = pl.NT < 8 ? 2 : 1;
    const int budget = 160 * 1024 / wg_per_cu - coop_extra_bytes(pl.NT);
    pa.nslot = std::max(2, std::min(budget / pa.slot_bytes, 6));
  }

  SolveArgs sa;
  memset(&sa, 0, sizeof(sa));
  sa.part_chunk_begin = d_pcb;
  sa.slab_H = slabH;
  sa.slab_g = slabg;
  sa.slab_ll = slabll;
  sa.theta = theta;
  sa.theta_prev = d_thprev;
  sa.delta_prev = d_dprev;
  sa.ll_prev = d_llprev;
  sa.phase = d_phase;
  sa.backtracks = d_bt;
  sa.iters = iters;
  sa.status = status;
  sa.counters = d_cnt;
  sa.sig_inv = sig_inv;
  sa.loglik = loglik;
  sa.P = P;
  sa.NT = pl.NT;
  sa.family = family;
  sa.tol = tol;
  sa.switch_tol = opt.switch_tol;
  sa.dm_prev = (double*)at(L.off_dmprev);
  sa.stall = (int32_t*)at(L.off_stall);
  // a stalled bf16-steered partition goes on with fp32-MFMA Hessians first
  sa.escalate_to = approx_prec == PREC_BF16 ? PHASE_F32X : PHASE_F64;

  const bool standardize = center != nullptr;
  StreamTimer timed{stream, opt.record_timing != 0};

  int32_t* h_cnt = pinned_staging(4 + 2 * (size_t)K);
  if (!h_cnt) {
    set_error("pinned host staging allocation failed");
    return DLSA_E_HIP;
  }

  const bool trace = getenv("DLSA_TRACE") != nullptr;
  int32_t* h_phase = h_cnt + 4;  // [K] phases (pinned: no staging copy per iteration)
  int32_t* h_route = h_phase + K;  // [K] phases with stale partitions marked (one launch)
  // exact passes on the int8 matrix cores (irls_oz_impl.hpp) unless DLSA_EXACT_FP64:
  // the first full-data bf16 pass records, per chunk and feature, max |x|; the
  // bf16 passes that follow an iteration with a partition near the switch
  // (counters[3], kOzNearTol) record max |sqrt(w) x| at the theta they saw
  // (snapshotted into theta_rec first); the exact passes of the final plan
  // take their digit scales from the partition's last records (a chunk with
  // no max |z| record -- zcolmax = +inf, theta_rec = 0 -- gets max |x| / 2)
  const bool use_oz = opt.exact_pass != DLSA_EXACT_FP64 && approx_prec == PREC_BF16 && oz_applies(pl.NT, p) &&
                      pl.max_chunk_rows <= kOzMaxRows;
  uint32_t* d_colmax = (uint32_t*)at(L.off_colmax);
  uint32_t* d_zcolmax = (uint32_t*)at(L.off_zcolmax);
  double* d_threc = (double*)at(L.off_threc);
  bool colmax_ready = false;
  bool near_switch = false;  // counters[3] of the last solve
  // per partition: the last approximate pass that processed it recorded max |z|
  // (so its exact pass starts from a record one small step away); a partition
  // lacking one runs its exact pass on the fp64 MFMA instead (a second launch
  // beside the int8 one, PHASE_F64_STALE): without a fresh record the digit
  // exponents fall back to max |x| / 2, which a column with large |x| at w ~ 0
  // (an outlier row) turns into ~1e-5 per-entry errors
  // (tests/test_gpu_ozaki.py::test_ozaki_polish_pass_per_entry)
  std::vector<char> zfresh((size_t)K, 0);
  // DLSA_OZ_ZREC=0 (knob builds, A/B only): no max |z| records, so no partition
  // is ever fresh and every exact pass runs on the fp64 MFMA (it no longer
  // measures round 3's "every exponent from max |x| / 2" int8 pass)
  const bool zrec = !(env_knob("DLSA_OZ_ZREC") && atoi(env_knob("DLSA_OZ_ZREC")) == 0);
  if (use_oz) {
    DLSA_HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)d_zcolmax, 0x7F800000u,
                                   (size_t)std::max(pl.n_chunks, 1) * pl.PP, stream));
    DLSA_HIP_TRY(hipMemsetAsync(d_threc, 0, 8LL * K * P, stream));
  }
  // one pass over the chunks of plan q whose partition is in phase ph:
  // exact (fp64 Hessian) passes by the per-wave kernel up to P = 128 and the
  // cooperative one above; approximate passes (PHASE_F32 at the fit's
  // approximate precision, PHASE_F32X at fp32) by the cooperative kernel
  // (full: q is the all-rows plan, whose chunks the digit scales describe)
  auto fused_pass = [&](int ph, const Plan& q, bool full, const std::vector<int64_t>& part_rows,
                        const int32_t* hph) -> hipError_t {
    const bool f64 = ph == PHASE_F64;
    const int prec = f64 ? PREC_F64 : (ph == PHASE_F32X ? PREC_F32 : approx_prec);
    pa.want_phase = ph;
    const bool wave = f64 && q.NT <= kWaveMaxNT;
    int n_fresh = 0, n_stale = 0;
    if (f64)
      for (int k = 0; k < K; ++k)
        if (hph[k] == PHASE_F64) (zfresh[k] ? n_fresh : n_stale)++;
    const bool oz = wave && use_oz && colmax_ready && full && n_fresh > 0;
    // int8 for the fresh partitions, fp64 MFMA for the stale ones: the stale
    // ones are marked PHASE_F64_STALE on the device for the int8 launch (which
    // skips them), then passed by the per-wave fp64 kernel, then restored
    const bool split = oz && n_stale > 0;
    if (split) {
      for (int k = 0; k < K; ++k)
        h_route[k] = (hph[k] == PHASE_F64 && !zfresh[k]) ? PHASE_F64_STALE : hph[k];
      hipError_t e = hipMemcpyAsync(d_phase, h_route, 4LL * K, hipMemcpyHostToDevice, stream);
      if (e != hipSuccess) return e;
      g_stats.oz_stale_partitions += n_stale;
    }
    // digit-scale records of a full-data bf16 pass: max |x| on the first,
    // max |z| near the switch
    const bool rec_x = use_oz && full && ph == PHASE_F32 && !colmax_ready;
    const bool rec_z = use_oz && full && ph == PHASE_F32 && near_switch && zrec;
    if (rec_z) {
      hipError_t e = launch_theta_snapshot(K, P, d_phase, PHASE_F32, theta, d_threc, stream);
      if (e != hipSuccess) return e;
    }
    hipError_t e = timed(f64 ? &g_stats.ms_pass_fp64 : &g_stats.ms_pass_fp32, [&] {
      PassArgs pc = pa;
      pc.colmax = (oz || rec_x) ? d_colmax : nullptr;
      pc.zcolmax = (oz || rec_z) ? d_zcolmax : nullptr;
      pc.theta_rec = d_threc;
      if (oz) {
        hipError_t eo = launch_irls_oz(pc, q.NT, standardize, family, q.n_chunks, stream);
        if (eo != hipSuccess || !split) return eo;
        PassArgs ps = pa;  // the stale partitions on the fp64 MFMA
        ps.want_phase = PHASE_F64_STALE;
        return launch_irls_wave(ps, q.NT, standardize, family, q.n_chunks, stream);
      }
      // OLS (one pass at theta = 0): X streamed into registers, no LDS ring.
      // Its buffer range and row offsets are 32-bit: a caller's rows_per_chunk
      // of >= 2^31 bytes per chunk takes the per-wave kernel instead
      if (f64 && family == FAMILY_GAUSSIAN && ols_stream_applies(q.NT) &&
          (int64_t)q.max_chunk_rows * p * 8 < (1LL << 31))
        return launch_ols_stream(pc, q.NT, standardize, q.n_chunks, stream);
      if (wave) return launch_irls_wave(pc, q.NT, standardize, family, q.n_chunks, stream);
      return launch_irls_coop(pc, q.NT, prec, standardize, family, q.n_chunks, stream);
    });
    if (split && e == hipSuccess)  // hph is the pinned readback, unchanged until the next sync
      e = hipMemcpyAsync(d_phase, hph, 4LL * K, hipMemcpyHostToDevice, stream);
    if (rec_x) colmax_ready = true;
    if (!f64)  // this pass's partitions moved on from their records unless it took one
      for (int k = 0; k < K; ++k)
        if (hph[k] == ph) zfresh[k] = rec_z;
    if (oz) g_stats.passes_oz++;
    if (f64) {
      g_stats.passes_fp64++;
      g_stats.rows_fp64 += phase_rows(part_rows, hph, ph);
    } else {
      g_stats.passes_fp32++;
      g_stats.rows_fp32 += phase_rows(part_rows, hph, ph);
      if (ph == PHASE_F32X) g_stats.passes_f32x++;
    }
    return e;
  };
  // The next iteration's approximate pass is enqueued before the host reads
  // this iteration's counters (DLSA_SPEC_PASS): a pass checks its partitions'
  // phases on the device, so one enqueued for partitions that have since
  // switched or finished runs as a no-op, and the GPU no longer idles through
  // every hand-back (hipStreamSynchronize's return, the host's decisions and
  // the next launch: 25-45 us per iteration).  The one decision
  // such a pass needs from those counters -- whether to record max |z| (a
  // partition near the switch, counters[3]) -- is taken on the device
  // (PassArgs::zrec_gate, the gated theta snapshot), and the host's
  // bookkeeping of the pass (zfresh, stats) runs after the read, from the
  // phases the pass saw.
  struct ReadEvent {  // the counters' copy of an iteration (destroyed on every return)
    hipEvent_t ev = nullptr;
    ~ReadEvent() {
      if (ev) (void)hipEventDestroy(ev);
    }
  } read_ev;
  if (DLSA_SPEC_PASS) DLSA_HIP_TRY(hipEventCreateWithFlags(&read_ev.ev, hipEventDisableTiming));
  auto spec_pass = [&](const Plan& q, bool full) -> hipError_t {
    pa.want_phase = PHASE_F32;
    const bool zg = use_oz && full && zrec;
    if (zg) {
      hipError_t e = launch_theta_snapshot(K, P, d_phase, PHASE_F32, theta, d_threc, stream, d_cnt + 3);
      if (e != hipSuccess) return e;
    }
    return timed(&g_stats.ms_pass_fp32, [&] {
      PassArgs pc = pa;
      pc.colmax = nullptr;
      pc.zcolmax = zg ? d_zcolmax : nullptr;
      pc.theta_rec = d_threc;
      pc.zrec_gate = zg ? d_cnt + 3 : nullptr;
      return launch_irls_coop(pc, q.NT, approx_prec, standardize, family, q.n_chunks, stream);
    });
  };
  int it = 0;
  for (size_t lvl = 0; lvl < plans.size(); ++lvl) {
    const Plan& q = plans[lvl];
    const bool final_level = lvl + 1 == plans.size();
    const std::vector<int64_t> part_rows = plan_part_rows(q, K);
    bool spec = false;  // this iteration's PHASE_F32 pass was enqueued before the last read
    DLSA_HIP_TRY(upload(q));
    if (lvl > 0) {  // re-enter every running partition
      DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
      DLSA_HIP_TRY(launch_level_reset(K, P, start_phase, d_phase, status, d_llprev, d_bt, theta,
                                      d_cnt, stream));
      DLSA_HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 16 + 4LL * K, hipMemcpyDeviceToHost, stream));
    } else {
      DLSA_HIP_TRY(hipMemcpyAsync(h_phase, d_phase, 4LL * K, hipMemcpyDeviceToHost, stream));
    }
    DLSA_HIP_TRY(hipStreamSynchronize(stream));
    if (lvl > 0)
      for (int ph = 0; ph < kRunPhases; ++ph) n_running[ph] = h_cnt[ph];
    sa.subsample = final_level ? 0 : 1;
    // the prefix MLE is ~sqrt(P/n) from the full one (max step ~0.35 entering
    // the full level at config 2), so a level need not converge: it stops at
    // a 0.2-relative step (warm_level_tol)
    sa.level_tol = warm_level_tol(true);
    sa.switch_tol = final_level ? opt.switch_tol : 0.0;
    const int it_end = it + iter_budget(final_level, it, max_iter);
    if (it_end <= it) continue;  // no budget left for this warm-start level
    DLSA_HIP_TRY(hipMemsetAsync(sa.dm_prev, 0, 8LL * K, stream));
    DLSA_HIP_TRY(hipMemsetAsync(sa.stall, 0, 4LL * K, stream));
    for (; it < it_end && running_total(n_running) > 0 && q.n_chunks > 0; ++it) {
      // approximate (bf16 or fp32), escalated fp32, then exact passes
      for (int ph : {PHASE_F32, PHASE_F32X, PHASE_F64}) {
        if (ph == PHASE_F32 && spec) {
          // enqueued before the last read: its bookkeeping, from the phases it saw
          if (n_running[ph] > 0) {
            const bool rz = use_oz && final_level && zrec && near_switch;  // the device's decision
            for (int k = 0; k < K; ++k)
              if (h_phase[k] == ph) zfresh[k] = rz;
            g_stats.passes_fp32++;
            g_stats.rows_fp32 += phase_rows(part_rows, h_phase, ph);
          }
          continue;
        }
        if (n_running[ph] == 0) continue;
        DLSA_HIP_TRY(fused_pass(ph, q, final_level, part_rows, h_phase));
      }
      DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
      DLSA_HIP_TRY(timed(&g_stats.ms_solve, [&] { return launch_newton_solve(sa, K, stream); }));
      // counters + phases in one copy (adjacent on both sides)
      DLSA_HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 16 + 4LL * K, hipMemcpyDeviceToHost, stream));
      // the next iteration's approximate pass, if this one had approximate
      // partitions and the next needs no first max |x| record (rec_x)
      spec = DLSA_SPEC_PASS && n_running[PHASE_F32] > 0 && it + 1 < it_end &&
             !(use_oz && final_level && !colmax_ready);
      if (spec) {
        // wait for the copy only: the pass runs on while the host decides
        DLSA_HIP_TRY(hipEventRecord(read_ev.ev, stream));
        DLSA_HIP_TRY(spec_pass(q, final_level));
        DLSA_HIP_TRY(hipEventSynchronize(read_ev.ev));
      } else {
        DLSA_HIP_TRY(hipStreamSynchronize(stream));
      }
      for (int ph = 0; ph < kRunPhases; ++ph) n_running[ph] = h_cnt[ph];
      near_switch = final_level && h_cnt[3] > 0;
      if (trace) DLSA_HIP_TRY(trace_iteration(K, P, theta, d_dprev, lvl, it, n_running));
    }
  }
  g_stats.iterations = it;
  // polish: partitions the budget left running (any phase) get one exact pass
  // at the theta they return; its X^T W X is published as Sig_inv, no step
  // (models.py:114,130 evaluate the weights at the coef sklearn stopped at)
  if (family == FAMILY_LOGISTIC && running_total(n_running) > 0 && pl.n_chunks > 0) {
    // (the final level's plan, pl, is on the device: it was the last uploaded)
    // a partition stopped in an approximate phase took a full step after its
    // last record: its polish pass cannot use that record
    for (int k = 0; k < K; ++k)
      if (h_phase[k] != PHASE_F64) zfresh[k] = 0;
    DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
    DLSA_HIP_TRY(launch_polish_mark(K, d_phase, status, d_cnt, stream));
    DLSA_HIP_TRY(hipMemcpyAsync(h_phase, d_phase, 4LL * K, hipMemcpyDeviceToHost, stream));
    DLSA_HIP_TRY(hipStreamSynchronize(stream));
    g_stats.polish_partitions = running_total(n_running);
    DLSA_HIP_TRY(fused_pass(PHASE_F64, plans.back(), true, plan_part_rows(pl, K), h_phase));
    sa.eval_only = 1;
    sa.subsample = 0;
    DLSA_HIP_TRY(timed(&g_stats.ms_solve, [&] { return launch_newton_solve(sa, K, stream); }));
    sa.eval_only = 0;
  }

  DLSA_HIP_TRY(launch_fit_finalize(K, P, theta, sig_inv, sig_inv_theta, status, stream));
  DLSA_HIP_TRY(hipStreamSynchronize(stream));
  g_stats.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                                               t_start)
                         .count();
  DLSA_HIP_TRY(timed.flush());
  return DLSA_OK;
}

// ---- categorical-code fit (cat_pass.hip) ---------------------------------
// level slots x replicas per factor of the numeric x dummy histograms before
// the LDS budget shrinks them (A/B builds: DLSA_CAT_ND_CAP)
#ifndef DLSA_CAT_ND_CAP
#define DLSA_CAT_ND_CAP 256
#endif
// LDS layout of the histograms: replicas so that a frequent level does not
// serialise the lanes of a wave on one address (nd: <= 128 slots per factor,
// pairs: <= 512 cells), shrunk until the workgroup fits 160 KB.
static bool cat_layout(CatArgs& a, const int32_t* levels) {
  const int Qw = (a.q + 1) | 1;
  a.nd_stride = Qw;
  // the exact-bucket kernel folds the intercept row into the histograms of the
  // factor with the most levels (its baseline is the rarest: fewest extra adds)
  a.fold = -1;
  if (cat_exact_bucket(a))
    for (int f = 0; f < a.F; ++f)
      if (a.fold < 0 || levels[f] > levels[a.fold]) a.fold = f;
  int nd_cap = DLSA_CAT_ND_CAP, pr_cap = 512;
  for (int attempt = 0; attempt < 12; ++attempt) {
    int64_t o = 0;
    for (int f = 0; f < a.F; ++f) {
      const int nl = levels[f] - 1;
      const int ns = nl + (f == a.fold ? 1 : 0);  // level slots per replica
      int R = 1;
      while (R < 16 && ns * R * 2 <= nd_cap) R *= 2;
      a.nlev[f] = nl;
      a.nd_lev[f] = ns;
      a.nd_rep[f] = R;
      a.nd_off[f] = (int32_t)o;
      o += (int64_t)R * ns * Qw;
    }
    for (int f = 0; f < a.F; ++f) {
      a.g_off[f] = (int32_t)o;
      o += (int64_t)a.nd_rep[f] * a.nd_lev[f];
    }
    for (int f = 0; f < a.F; ++f)
      for (int g = f + 1; g < a.F; ++g) {
        const int pi = f * a.F - f * (f + 1) / 2 + (g - f - 1);
        const int cells = a.nlev[f] * a.nlev[g];
        int R = 1;
        while (R < 8 && cells * R * 2 <= pr_cap) R *= 2;
        a.pr_rep[pi] = R;
        a.pr_off[pi] = (int32_t)o;
        o += (int64_t)R * cells;
      }
    a.hist_doubles = (int32_t)std::min<int64_t>(o, INT32_MAX);
    if (cat_lds_bytes(a) + kCatStaticLds <= 160 * 1024) return true;
    if (nd_cap == 1 && pr_cap == 1) break;
    nd_cap = std::max(1, nd_cap / 2);
    pr_cap = std::max(1, pr_cap / 2);
  }
  return false;
}

static int fit_categorical(const double* Xn, const uint8_t* codes, const double* y,
                           const int64_t* offsets, int32_t K, int32_t q, int32_t F,
                           const int32_t* levels, int32_t fit_intercept, const double* center,
                           const double* scale, int32_t max_iter, double tol, double* theta,
                           double* sig_inv, double* sig_inv_theta, double* loglik, int32_t* iters,
                           int32_t* status, const dlsa_fit_options* opt_in, void* stream_) {
  const auto t_start = std::chrono::steady_clock::now();
  g_last_error.clear();
  memset(&g_stats, 0, sizeof(g_stats));
  hipStream_t stream = (hipStream_t)stream_;
  dlsa_fit_options opt;
  if (opt_in)
    opt = *opt_in;
  else
    dlsa_fit_options_default(&opt);
  int rc = check_offsets(offsets, K);
  if (rc != DLSA_OK) return rc;
  if (q < 0 || F < 0 || F > kCatMaxFactors || (F > 0 && !levels)) {
    set_error("need 0 <= q, 0 <= F <= 16 and a host levels[F] array");
    return DLSA_E_INVALID;
  }
  int D = 0;
  for (int f = 0; f < F; ++f) {
    if (levels[f] < 1 || levels[f] > 256) {
      set_error("levels[" + std::to_string(f) + "] must be in 1..256 (uint8 codes)");
      return DLSA_E_INVALID;
    }
    D += levels[f] - 1;
  }
  const int ic = fit_intercept ? 1 : 0;
  const int P = ic + q + D;
  if (P < 1 || P > DLSA_MAX_P_FUSED || ic + q > kCatQMax) {
    set_error("categorical fit needs 1 <= P = intercept + q + sum(levels - 1) <= " +
              std::to_string(DLSA_MAX_P_FUSED) + " and intercept + q <= " +
              std::to_string(kCatQMax) + " (got P = " + std::to_string(P) + ")");
    return DLSA_E_UNSUPPORTED;
  }
  if ((center == nullptr) != (scale == nullptr)) {
    set_error("center and scale must both be given or both be NULL");
    return DLSA_E_INVALID;
  }
  if (!theta || !sig_inv || !sig_inv_theta || !loglik || !iters || !status) {
    set_error("null output pointer");
    return DLSA_E_INVALID;
  }
  const int64_t n_total = offsets[K];
  if (n_total > 0 && (!y || (q > 0 && !Xn) || (F > 0 && !codes))) {
    set_error("null Xn, codes or y");
    return DLSA_E_INVALID;
  }
  if (max_iter < 1) max_iter = 1;
  if (!(tol > 0)) tol = 1e-10;

  CatArgs ca;
  memset(&ca, 0, sizeof(ca));
  ca.q = q;
  ca.F = F;
  ca.P = P;
  ca.intercept = ic;
  int d = ic + q;
  for (int f = 0; f < F; ++f) {
    ca.doff[f] = d;
    d += levels[f] - 1;
  }
  if (!cat_layout(ca, levels)) {
    set_error("categorical histograms do not fit the 160 KB LDS of a workgroup (P = " +
              std::to_string(P) + ")");
    return DLSA_E_UNSUPPORTED;
  }

  // chunks: one workgroup per CU at this LDS size, so a launch should be
  // whole rounds of 256 workgroups: ~512 chunks, split evenly per partition
  // (a ceil-rounded n/512 gave 5 chunks per config-3 partition -> 640 chunks,
  // 3 rounds of which the last is half empty)
  auto cat_rpc = [&](double frac, int64_t min_rows) {
    if (opt.rows_per_chunk > 0) return (int)opt.rows_per_chunk;
    int64_t nmax = 0;
    for (int k = 0; k < K; ++k)
      nmax = std::max(nmax, rows_used(offsets[k + 1] - offsets[k], frac, min_rows));
    const int64_t per = std::max<int64_t>(1, 512 / std::max(K, 1));
    return (int)std::max<int64_t>(1024, std::min<int64_t>((nmax + per - 1) / per, 1 << 24));
  };
  // warm-start level (a 1/16 prefix of every partition, to a 0.2-relative
  // step) only for partitions of >= 2^19 rows on average: every categorical
  // pass is exact, so on small partitions the prefix passes' launches and host
  // round trips cost more than the full pass they save (1.5e7 rows in 128
  // partitions: 11.2 ms per fit without, 14.9 with, profiles r02), on large
  // ones they save a full pass (config 3, 1.2e8 rows in 120 partitions: 37.2
  // vs 38.7 ms per step, 7 vs 5 passes of which 4 vs 5 full,
  // profiles/r04n_cat_warm_start_ab.txt).  DLSA_WARM_START overrides.
  std::vector<Plan> plans;
  opt.warm_start = opt.warm_start && K > 0 && n_total / K >= (int64_t(1) << 19);
  if (const char* e = env_knob("DLSA_WARM_START")) opt.warm_start = atoi(e);
  if (opt.warm_start) {
    const int64_t min_rows = std::max<int64_t>(2048, level_rows_per_param() * P);
    for (double frac : warm_level_fracs(true)) {
      Plan qn;
      const int64_t lr = level_rows(offsets, K, frac, min_rows);
      make_plan(offsets, K, P - ic, ic, cat_rpc(frac, min_rows), qn, frac, min_rows);
      if (lr <= n_total / 2 && qn.n_chunks > 0) plans.push_back(std::move(qn));
    }
  }
  {
    Plan full;
    make_plan(offsets, K, P - ic, ic, cat_rpc(1.0, 0), full);
    plans.push_back(std::move(full));
  }
  const Plan& pl = plans.back();
  int max_chunks = 0;
  for (const Plan& qn : plans) max_chunks = std::max(max_chunks, qn.n_chunks);
  Plan sizing = pl;
  sizing.n_chunks = max_chunks;
  const Layout L = make_layout(sizing, K);
  const int64_t off_counts = align_up(L.total, 256);
  const int64_t off_bad = align_up(off_counts + 4LL * std::max(pl.n_chunks, 1) * std::max(D, 1), 256);
  const int64_t off_badp = align_up(off_bad + 4LL * std::max(pl.n_chunks, 1), 256);
  const int64_t off_colmax = align_up(off_badp + 4LL * K, 256);
  const int64_t off_hs = align_up(off_colmax + 8LL * kCatQMax * std::max(pl.n_chunks, 1), 256);
  const int64_t total = align_up(off_hs + 8LL * (kCatQMax + 2) * K, 256);
  g_stats.n_chunks = pl.n_chunks;

  char* ws = (char*)opt.workspace;
  bool owned = false;
  if (!ws || opt.workspace_bytes < total) {
    DLSA_HIP_TRY(hipMallocAsync((void**)&ws, total, stream));
    owned = true;
  }
  struct Free {
    char* p;
    bool own;
    hipStream_t s;
    ~Free() {
      if (own && p) (void)hipFreeAsync(p, s);
    }
  } freer{ws, owned, stream};
  auto at = [&](int64_t off) { return (void*)(ws + off); };
  int64_t* d_row0 = (int64_t*)at(L.off_row0);
  int32_t* d_rows = (int32_t*)at(L.off_rows);
  int32_t* d_part = (int32_t*)at(L.off_part);
  int32_t* d_pcb = (int32_t*)at(L.off_pcb);
  int64_t* d_offsets = (int64_t*)at(L.off_offsets);
  int32_t* d_phase = (int32_t*)at(L.off_phase);
  int32_t* d_bt = (int32_t*)at(L.off_bt);
  double* d_llprev = (double*)at(L.off_llprev);
  int32_t* d_cnt = (int32_t*)at(L.off_counters);
  int32_t* d_counts = (int32_t*)at(off_counts);
  int32_t* d_bad = (int32_t*)at(off_bad);
  int32_t* d_badp = (int32_t*)at(off_badp);
  double* d_colmax = (double*)at(off_colmax);
  double* d_hs = (double*)at(off_hs);

  auto upload = [&](const Plan& qn) -> hipError_t {
    return upload_plan_tables(qn, K, d_row0, d_rows, d_part, d_pcb, stream);
  };
  {
    // every level is uploaded once, the final plan twice (presence pass, then
    // again after the warm-start levels)
    size_t need = staged_bytes(8 * ((size_t)K + 1)) + plan_staged_bytes(pl, K) +
                  staged_bytes(8 * ((size_t)kCatQMax + 2) * K);  // + the grids
    for (const Plan& qn : plans) need += plan_staged_bytes(qn, K);
    DLSA_HIP_TRY(pinned_arena_reserve(need));
  }
  DLSA_HIP_TRY(staged_upload(d_offsets, offsets, 8LL * (K + 1), stream));
  DLSA_HIP_TRY(launch_fit_init(d_offsets, K, P, PHASE_F64, theta, d_phase, d_bt, iters, status,
                               d_llprev, sig_inv, loglik, stream));

  ca.Xn = Xn;
  ca.codes = codes;
  ca.y = y;
  ca.chunk_row0 = d_row0;
  ca.chunk_rows = d_rows;
  ca.chunk_part = d_part;
  ca.phase = d_phase;
  ca.theta = theta;
  ca.center = center;
  ca.scale = scale;
  ca.slab_H = (double*)at(L.off_slabH);
  ca.slab_g = (double*)at(L.off_slabg);
  ca.slab_ll = (double*)at(L.off_slabll);
  ca.NT = pl.NT;
  ca.want_phase = PHASE_F64;

  // level presence over all rows: partitions missing a level -> zero frame;
  // invalid codes fail the call.  The same pass takes max |x_i| per column for
  // the fixed-point grids of the histograms (cat_pass.hip).
  // counters + phases in pinned staging (h_phase = h_cnt + 4, like d_cnt / d_phase)
  int32_t* h_cnt = pinned_staging(4 + (size_t)K);
  if (!h_cnt) {
    set_error("pinned host staging allocation failed");
    return DLSA_E_HIP;
  }
  int32_t* h_phase = h_cnt + 4;
  std::vector<int32_t> h_badp(K, 0);
  std::vector<double> h_colmax((size_t)kCatQMax * std::max(pl.n_chunks, 1), 0.0);
  DLSA_HIP_TRY(upload(pl));
  DLSA_HIP_TRY(launch_cat_presence(ca, pl.n_chunks, d_counts, d_bad, d_colmax, stream));
  if (pl.n_chunks > 0)
    DLSA_HIP_TRY(hipMemcpyAsync(h_colmax.data(), d_colmax, 8LL * kCatQMax * pl.n_chunks,
                                hipMemcpyDeviceToHost, stream));
  if (D > 0) {
    DLSA_HIP_TRY(launch_cat_mark(ca, d_pcb, d_counts, d_bad, K, d_phase, status, d_badp, stream));
    DLSA_HIP_TRY(hipMemcpyAsync(h_badp.data(), d_badp, 4LL * K, hipMemcpyDeviceToHost, stream));
  }
  DLSA_HIP_TRY(hipMemcpyAsync(h_phase, d_phase, 4LL * K, hipMemcpyDeviceToHost, stream));
  DLSA_HIP_TRY(hipStreamSynchronize(stream));
  std::vector<double> h_hs;  // the grids (staged into the pinned arena on upload)
  {
    // fixed-point grids: 2^E with |term| * 2^E * max(rows of a chunk, 1024) <= 2^60,
    // so a bin's sum stays in int64 and every term below 2^50 (the kernel's
    // 1.5 * 2^52 rounding needs |term| < 2^51)
    int64_t rmax = 1024;
    for (const Plan& qn : plans)
      for (int c = 0; c < qn.n_chunks; ++c) rmax = std::max<int64_t>(rmax, qn.chunk_rows[c]);
    auto grid = [&](double bound) {  // bound: max |term|
      if (!(bound > 0) || !std::isfinite(bound)) bound = 1.0;
      const int e = (int)std::floor(60.0 - std::log2(bound * (double)rmax));
      return std::ldexp(1.0, std::max(-900, std::min(900, e)));
    };
    // per partition (its chunks of the full plan cover all its rows, so the
    // bound holds for every warm-start level's chunks too): an outlier row
    // coarsens only its own partition's grid
    std::vector<double> hc(q, 0.0), hs(q, 1.0);
    if (center && q > 0) {  // the kernel sums w (x - c) / s
      DLSA_HIP_TRY(hipMemcpy(hc.data(), center, 8LL * q, hipMemcpyDeviceToHost));
      DLSA_HIP_TRY(hipMemcpy(hs.data(), scale, 8LL * q, hipMemcpyDeviceToHost));
    }
    h_hs.assign((size_t)K * (kCatQMax + 2), 1.0);
    for (int k = 0; k < K; ++k) {
      double* o = h_hs.data() + (size_t)k * (kCatQMax + 2);
      o[0] = grid(0.25);  // w = mu (1 - mu) <= 1/4; pair cells
      o[1] = grid(1.0);   // |y - mu| <= 1
      for (int j = 0; j < q; ++j) {
        double m = 0.0;
        for (int c = pl.part_chunk_begin[k]; c < pl.part_chunk_begin[k + 1]; ++c)
          m = std::max(m, h_colmax[(size_t)c * kCatQMax + j]);
        if (center) m = (m + std::fabs(hc[j])) / std::fabs(hs[j]);
        o[2 + j] = grid(0.25 * m);
      }
    }
    DLSA_HIP_TRY(staged_upload(d_hs, h_hs.data(), 8LL * (kCatQMax + 2) * K, stream));
    ca.hscale = d_hs;
  }
  for (int k = 0; k < K; ++k)
    if (h_badp[k]) {
      set_error("partition " + std::to_string(k) + ": " + std::to_string(h_badp[k]) +
                " level codes >= levels[f]");
      return DLSA_E_INVALID;
    }
  int n_running = 0;
  for (int k = 0; k < K; ++k) n_running += h_phase[k] == PHASE_F64;

  SolveArgs sa;
  memset(&sa, 0, sizeof(sa));
  sa.part_chunk_begin = d_pcb;
  sa.slab_H = ca.slab_H;
  sa.slab_g = ca.slab_g;
  sa.slab_ll = ca.slab_ll;
  sa.theta = theta;
  sa.theta_prev = (double*)at(L.off_thprev);
  sa.delta_prev = (double*)at(L.off_dprev);
  sa.ll_prev = d_llprev;
  sa.phase = d_phase;
  sa.backtracks = d_bt;
  sa.iters = iters;
  sa.status = status;
  sa.counters = d_cnt;
  sa.sig_inv = sig_inv;
  sa.loglik = loglik;
  sa.P = P;
  sa.NT = pl.NT;
  sa.family = FAMILY_LOGISTIC;
  sa.tol = tol;
  sa.dm_prev = (double*)at(L.off_dmprev);
  sa.stall = (int32_t*)at(L.off_stall);
  sa.escalate_to = PHASE_F64;  // every categorical pass is exact

  const bool standardize = center != nullptr;
  StreamTimer timed{stream, opt.record_timing != 0};
  const bool trace = getenv("DLSA_TRACE") != nullptr;

  int it = 0;
  for (size_t lvl = 0; lvl < plans.size(); ++lvl) {
    const Plan& qn = plans[lvl];
    const bool final_level = lvl + 1 == plans.size();
    const std::vector<int64_t> part_rows = plan_part_rows(qn, K);
    DLSA_HIP_TRY(upload(qn));
    if (lvl > 0) {
      DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
      DLSA_HIP_TRY(launch_level_reset(K, P, PHASE_F64, d_phase, status, d_llprev, d_bt, theta,
                                      d_cnt, stream));
      DLSA_HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 16 + 4LL * K, hipMemcpyDeviceToHost, stream));
      DLSA_HIP_TRY(hipStreamSynchronize(stream));
      n_running = h_cnt[0] + h_cnt[1] + h_cnt[2];
    }
    sa.subsample = final_level ? 0 : 1;
    sa.level_tol = warm_level_tol(true);
    sa.switch_tol = 0.0;
    const int it_end = it + iter_budget(final_level, it, max_iter);
    if (it_end <= it) continue;  // no budget left for this warm-start level
    for (; it < it_end && n_running > 0 && qn.n_chunks > 0; ++it) {
      DLSA_HIP_TRY(timed(&g_stats.ms_pass_fp64,
                         [&] { return launch_cat_pass(ca, standardize, qn.n_chunks, stream); }));
      g_stats.passes_fp64++;
      g_stats.rows_fp64 += phase_rows(part_rows, h_phase, PHASE_F64);
      DLSA_HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, stream));
      DLSA_HIP_TRY(timed(&g_stats.ms_solve, [&] { return launch_newton_solve(sa, K, stream); }));
      DLSA_HIP_TRY(hipMemcpyAsync(h_cnt, d_cnt, 16 + 4LL * K, hipMemcpyDeviceToHost, stream));
      DLSA_HIP_TRY(hipStreamSynchronize(stream));
      n_running = h_cnt[0] + h_cnt[1] + h_cnt[2];
      int nr[kRunPhases] = {h_cnt[0], h_cnt[1], h_cnt[2]};
      if (trace) DLSA_HIP_TRY(trace_iteration(K, P, theta, sa.delta_prev, lvl, it, nr));
    }
  }
  g_stats.iterations = it;
  // polish: Sig_inv of a partition the budget left running at the theta it
  // returns (one more exact pass, no step; see fit_impl)
  if (n_running > 0 && pl.n_chunks > 0) {
    if (plans.size() > 1) DLSA_HIP_TRY(upload(pl));
    DLSA_HIP_TRY(timed(&g_stats.ms_pass_fp64,
                       [&] { return launch_cat_pass(ca, standardize, pl.n_chunks, stream); }));
    g_stats.passes_fp64++;
    g_stats.rows_fp64 += phase_rows(plan_part_rows(pl, K), h_phase, PHASE_F64);
    g_stats.polish_partitions = n_running;
    sa.eval_only = 1;
    sa.subsample = 0;
    DLSA_HIP_TRY(timed(&g_stats.ms_solve, [&] { return launch_newton_solve(sa, K, stream); }));
    sa.eval_only = 0;
  }
  DLSA_HIP_TRY(launch_fit_finalize(K, P, theta, sig_inv, sig_inv_theta, status, stream));
  DLSA_HIP_TRY(hipStreamSynchronize(stream));
  g_stats.ms_total =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start)
          .count();
  DLSA_HIP_TRY(timed.flush());
  return DLSA_OK;
}

}  // namespace dlsa

extern "C" {

int dlsa_logistic_fit_batched_ex(const double* X, const double* y, const int64_t* offsets,
                                 int32_t K, int32_t p, int32_t fit_intercept,
                                 const double* center, const double* scale, int32_t max_iter,
                                 double tol, double* theta, double* sig_inv,
                                 double* sig_inv_theta, double* loglik, int32_t* iters,
                                 int32_t* status, const dlsa_fit_options* opt, void* stream) {
  return fit_impl(FAMILY_LOGISTIC, X, y, offsets, K, p, fit_intercept, center, scale, max_iter,
                  tol, theta, sig_inv, sig_inv_theta, loglik, iters, status, opt, stream);
}

int dlsa_logistic_fit_categorical(const double* Xn, const uint8_t* codes, const double* y,
                                  const int64_t* offsets, int32_t K, int32_t q, int32_t F,
                                  const int32_t* levels, int32_t fit_intercept,
                                  const double* center, const double* scale, int32_t max_iter,
                                  double tol, double* theta, double* sig_inv,
                                  double* sig_inv_theta, double* loglik, int32_t* iters,
                                  int32_t* status, const dlsa_fit_options* opt, void* stream) {
  return fit_categorical(Xn, codes, y, offsets, K, q, F, levels, fit_intercept, center, scale,
                         max_iter, tol, theta, sig_inv, sig_inv_theta, loglik, iters, status, opt,
                         stream);
}

int dlsa_ols_fit_batched(const double* X, const double* y, const int64_t* offsets, int32_t K,
                         int32_t p, int32_t fit_intercept, const double* center,
                         const double* scale, double* theta, double* sig_inv,
                         double* sig_inv_theta, double* rss, int32_t* status,
                         const dlsa_fit_options* opt, void* stream) {
  dlsa_fit_options o;
  if (opt)
    o = *opt;
  else
    dlsa_fit_options_default(&o);
  o.hessian_mode = DLSA_HESSIAN_FP64;
  // the iteration count is always 1 for OLS and not part of this ABI: give
  // the driver a throw-away device array for it
  int32_t* d_iters = nullptr;
  hipStream_t s = (hipStream_t)stream;
  if (K > 0) {
    hipError_t e = hipMallocAsync((void**)&d_iters, sizeof(int32_t) * K, s);
    if (e != hipSuccess) {
      set_error(std::string("hipMallocAsync: ") + hipGetErrorString(e));
      return DLSA_E_HIP;
    }
  }
  const int rc = fit_impl(FAMILY_GAUSSIAN, X, y, offsets, K, p, fit_intercept, center, scale, 1,
                          1.0, theta, sig_inv, sig_inv_theta, rss, d_iters, status, &o, stream);
  if (d_iters) (void)hipFreeAsync(d_iters, s);
  return rc;
}

int dlsa_logistic_fit_batched(const double* X, const double* y, const int64_t* offsets,
                              int32_t K, int32_t p, int32_t fit_intercept, const double* center,
                              const double* scale, int32_t max_iter, double tol, double* theta,
                              double* sig_inv, double* sig_inv_theta, double* loglik,
                              int32_t* iters, int32_t* status, void* stream) {
  return dlsa_logistic_fit_batched_ex(X, y, offsets, K, p, fit_intercept, center, scale,
                                      max_iter, tol, theta, sig_inv, sig_inv_theta, loglik,
                                      iters, status, nullptr, stream);
}

int dlsa_logistic_loglik_batched(const double* X, const double* y, const int64_t* offsets,
                                 int32_t K, int32_t p, int32_t fit_intercept,
                                 const double* center, const double* scale,
                                 const double* betas, int32_t n_beta, double* loglik,
                                 void* stream_) {
  g_last_error.clear();
  hipStream_t stream = (hipStream_t)stream_;
  int rc = check_offsets(offsets, K);
  if (rc != DLSA_OK) return rc;
  const int P = p + (fit_intercept ? 1 : 0);
  if (p < 0 || P < 1 || P > 512 || n_beta < 1 || n_beta > 16 || !betas || !loglik ||
      (center == nullptr) != (scale == nullptr)) {
    set_error("dlsa_logistic_loglik_batched: invalid arguments (1 <= P <= 512, 1 <= n_beta <= 16)");
    return DLSA_E_INVALID;
  }
  const int64_t n_total = offsets[K];
  if (n_total > 0 && (!X || !y)) {
    set_error("null X or y");
    return DLSA_E_INVALID;
  }
  Plan pl;
  make_plan(offsets, K, p, fit_intercept, 0, pl);
  const int nc = std::max(pl.n_chunks, 1);
  const int64_t bytes = align_up(8LL * nc, 256) + 3 * align_up(4LL * nc, 256) +
                        align_up(4LL * (K + 1), 256) + align_up(8LL * nc * n_beta, 256);
  char* ws = nullptr;
  DLSA_HIP_TRY(hipMallocAsync((void**)&ws, bytes, stream));
  struct Free {
    char* p;
    hipStream_t s;
    ~Free() {
      if (p) (void)hipFreeAsync(p, s);
    }
  } freer{ws, stream};
  int64_t o = 0;
  int64_t* d_row0 = (int64_t*)(ws + o);
  o += align_up(8LL * nc, 256);
  int32_t* d_rows = (int32_t*)(ws + o);
  o += align_up(4LL * nc, 256);
  int32_t* d_part = (int32_t*)(ws + o);
  o += align_up(4LL * nc, 256);
  int32_t* d_pcb = (int32_t*)(ws + o);
  o += align_up(4LL * (K + 1), 256);
  double* d_partial = (double*)(ws + o);
  if (pl.n_chunks > 0) {
    DLSA_HIP_TRY(hipMemcpyAsync(d_row0, pl.chunk_row0.data(), 8LL * pl.n_chunks,
                                hipMemcpyHostToDevice, stream));
    DLSA_HIP_TRY(hipMemcpyAsync(d_rows, pl.chunk_rows.data(), 4LL * pl.n_chunks,
                                hipMemcpyHostToDevice, stream));
    DLSA_HIP_TRY(hipMemcpyAsync(d_part, pl.chunk_part.data(), 4LL * pl.n_chunks,
                                hipMemcpyHostToDevice, stream));
  }
  DLSA_HIP_TRY(hipMemcpyAsync(d_pcb, pl.part_chunk_begin.data(), 4LL * (K + 1),
                              hipMemcpyHostToDevice, stream));
  if (pl.n_chunks > 0) {
    EvalArgs ea;
    memset(&ea, 0, sizeof(ea));
    ea.X = X;
    ea.y = y;
    ea.chunk_row0 = d_row0;
    ea.chunk_rows = d_rows;
    ea.chunk_part = d_part;
    ea.center = center;
    ea.scale = scale;
    ea.betas = betas;
    ea.partial = d_partial;
    const uintptr_t xend = (uintptr_t)(X + n_total * (int64_t)p);
    ea.x_last16 = ((xend + 15) & ~(uintptr_t)15) - 16;
    ea.y_last4 = (uintptr_t)(y + n_total) - 4;
    ea.p = p;
    ea.P = P;
    ea.intercept = fit_intercept ? 1 : 0;
    ea.nbeta = n_beta;
    ea.slot_bytes = eval_slot_bytes(p);
    const int PM = ((P + 7) / 8) * 8;
    const int budget = 160 * 1024 - (n_beta * PM + 2 * PM + 64) * 8;
    ea.nslot = std::max(2, std::min(budget / ea.slot_bytes, 6));
    DLSA_HIP_TRY(launch_loglik_eval(ea, pl.n_chunks, stream));
  }
  DLSA_HIP_TRY(launch_loglik_reduce(d_partial, d_pcb, K, n_beta, loglik, stream));
  DLSA_HIP_TRY(hipStreamSynchronize(stream));
  return DLSA_OK;
}

int dlsa_partition_rows(const int32_t* part_id, int64_t n, int32_t K, int32_t n_arrays,
                        const void* const* src, void* const* dst, const int64_t* row_bytes,
                        int64_t* offsets, int64_t* order, void* stream_) {
  g_last_error.clear();
  hipStream_t stream = (hipStream_t)stream_;
  if (K < 1 || K > kPartMaxK || n < 0 || n_arrays < 0 || n_arrays > kPartMaxArrays ||
      !offsets || (n_arrays > 0 && (!src || !dst || !row_bytes))) {
    set_error("dlsa_partition_rows: need 1 <= K <= " + std::to_string(kPartMaxK) +
              ", 0 <= n_arrays <= " + std::to_string(kPartMaxArrays) +
              ", host src/dst/row_bytes arrays and a host offsets[K+1]");
    return DLSA_E_INVALID;
  }
  for (int a = 0; a < n_arrays; ++a)
    if (row_bytes[a] < 1 || (n > 0 && (!src[a] || !dst[a]))) {
      set_error("dlsa_partition_rows: array " + std::to_string(a) + " has no rows or pointers");
      return DLSA_E_INVALID;
    }
  if (n == 0) {
    for (int k = 0; k <= K; ++k) offsets[k] = 0;
    return DLSA_OK;
  }
  if (!part_id) {
    set_error("dlsa_partition_rows: null part_id");
    return DLSA_E_INVALID;
  }
  // ~2048 blocks of input rows (block order = input order: stable)
  const int64_t rpb = std::max<int64_t>(kPartSubRows, (n + 2047) / 2048);
  const int nb = (int)((n + rpb - 1) / rpb);
  const int64_t off_counts = 0;
  const int64_t off_bad = align_up(4LL * nb * K, 256);
  const int64_t off_tot = align_up(off_bad + 4LL * nb, 256);
  const int64_t off_offs = align_up(off_tot + 8LL * K, 256);
  const int64_t total = align_up(off_offs + 8LL * (K + 1), 256);
  char* ws = nullptr;
  DLSA_HIP_TRY(hipMallocAsync((void**)&ws, total, stream));
  struct Free {
    char* p;
    hipStream_t s;
    ~Free() {
      if (p) (void)hipFreeAsync(p, s);
    }
  } freer{ws, stream};
  int32_t* counts = (int32_t*)(ws + off_counts);
  int32_t* bad = (int32_t*)(ws + off_bad);
  int64_t* totals = (int64_t*)(ws + off_tot);
  int64_t* offs_dev = (int64_t*)(ws + off_offs);
  DLSA_HIP_TRY(launch_partition_rows(part_id, n, K, rpb, nb, counts, bad, totals, offs_dev,
                                     stream));
  std::vector<int32_t> h_bad(nb);
  DLSA_HIP_TRY(hipMemcpyAsync(h_bad.data(), bad, 4LL * nb, hipMemcpyDeviceToHost, stream));
  DLSA_HIP_TRY(hipMemcpyAsync(offsets, offs_dev, 8LL * (K + 1), hipMemcpyDeviceToHost, stream));
  DLSA_HIP_TRY(hipStreamSynchronize(stream));
  int64_t nbad = 0;
  for (int b = 0; b < nb; ++b) nbad += h_bad[b];
  if (nbad) {
    set_error("dlsa_partition_rows: " + std::to_string(nbad) + " partition ids outside [0, K)");
    return DLSA_E_INVALID;
  }
  for (int k = 0; k < K; ++k)
    if (offsets[k + 1] - offsets[k] > INT32_MAX) {
      set_error("dlsa_partition_rows: a partition has more than 2^31 - 1 rows");
      return DLSA_E_UNSUPPORTED;
    }
  DLSA_HIP_TRY(launch_partition_scatter(part_id, n, K, rpb, nb, counts, offs_dev, src, dst,
                                        row_bytes, n_arrays, order, stream));
  DLSA_HIP_TRY(hipStreamSynchronize(stream));
  return DLSA_OK;
}

int dlsa_reduce_partitions(const double* sig_inv, const double* sig_inv_theta,
                           const double* theta, int32_t K, int32_t p, double* out,
                           void* stream) {
  g_last_error.clear();
  if (K < 1 || p < 1 || !sig_inv || !sig_inv_theta || !theta || !out) {
    set_error("dlsa_reduce_partitions: invalid arguments");
    return DLSA_E_INVALID;
  }
  DLSA_HIP_TRY(launch_reduce_partitions(sig_inv, sig_inv_theta, theta, K, p, out,
                                        (hipStream_t)stream));
  return DLSA_OK;
}

int dlsa_column_moments(const double* X, int64_t n, int32_t p, double* out, void* stream_) {
  g_last_error.clear();
  if (n < 0 || p < 1 || (n > 0 && !X) || !out) {
    set_error("dlsa_column_moments: invalid arguments");
    return DLSA_E_INVALID;
  }
  hipStream_t stream = (hipStream_t)stream_;
  int G = 1;
  int64_t rpr = 1;
  column_moments_plan(n, p, &G, &rpr);
  double* ws = nullptr;
  DLSA_HIP_TRY(hipMallocAsync((void**)&ws, sizeof(double) * (5LL * G + 5) * p, stream));
  const hipError_t e = launch_column_moments(X, n, p, out, ws, G, rpr, stream);
  const hipError_t f = hipFreeAsync(ws, stream);
  DLSA_HIP_TRY(e);
  DLSA_HIP_TRY(f);
  return DLSA_OK;
}

int dlsa_simulate_logistic(double* X, double* y, int64_t n, int32_t p, uint64_t seed,
                           int64_t row0, void* stream) {
  g_last_error.clear();
  if (n < 0 || p < 1 || (n > 0 && (!X || !y))) {
    set_error("dlsa_simulate_logistic: invalid arguments");
    return DLSA_E_INVALID;
  }
  DLSA_HIP_TRY(launch_simulate(X, y, n, p, seed, row0, (hipStream_t)stream));
  return DLSA_OK;
}

}  // extern "C"

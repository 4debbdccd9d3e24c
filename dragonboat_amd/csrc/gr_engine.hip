// gr_engine.hip — libgpuraft.so: the C-ABI declared in include/gpuraft.h, the
// boundary passes (gr_io.h) and the pass launcher; the step kernels themselves
// are in gr_kernels.h, one translation unit per slot count (gr_kernels_s*.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>


#include "gr_host.h"
#include "gr_io.h"
#include "gr_kernels.h"
#include "gpuraft_wire.h"

namespace gr {

#define GR_EXTERN_SLOTS(SS)                                                                                  \
  extern template hipError_t launch<SS>(const StepParams&, uint32_t*, uint32_t*, uint32_t, uint32_t, hipStream_t, \
                                        const PassTiming*, bool);
GR_EXTERN_SLOTS(1)
GR_EXTERN_SLOTS(3)
GR_EXTERN_SLOTS(5)
GR_EXTERN_SLOTS(8)
#ifdef GR_COVERAGE
extern template hipError_t cover_read<1>(uint64_t*);
extern template hipError_t cover_read<3>(uint64_t*);
extern template hipError_t cover_read<5>(uint64_t*);
extern template hipError_t cover_read<8>(uint64_t*);
#endif

// tick_lanes: launch the tick kernel (some lane may carry ticks or a ReadIndex).
static hipError_t launch_slots(uint32_t S, const StepParams& kp, uint32_t* bail_list, uint32_t* counters,
                               uint32_t list_cap, uint32_t parity, hipStream_t s, const PassTiming* t,
                               bool tick_lanes = true) {
  switch (S) {
    case 1: return launch<1>(kp, bail_list, counters, list_cap, parity, s, t, tick_lanes);
    case 3: return launch<3>(kp, bail_list, counters, list_cap, parity, s, t, tick_lanes);
    case 5: return launch<5>(kp, bail_list, counters, list_cap, parity, s, t, tick_lanes);
    case 8: return launch<8>(kp, bail_list, counters, list_cap, parity, s, t, tick_lanes);
  }
  return hipErrorInvalidValue;
}

static uint32_t instantiated_slots(uint32_t want) {
  if (want <= 1) return 1;
  if (want <= 3) return 3;
  if (want <= 5) return 5;
  if (want <= GR_SMAX) return GR_SMAX;  // wide groups (e.g. 5 voters + 2 observers): leaders take the general lane
  return 0;
}

}  // namespace gr

using namespace gr;
using namespace gr::host;

struct gr_engine {
  gr_config cfg{};
  uint32_t S = 0;
  uint32_t cap = 0;  // padded slot capacity (row stride)
  hipStream_t stream = nullptr;

  StateBase st{};
  LaneBase ln{};
  uint64_t* stats = nullptr;
  uint32_t stats_rows = 0;
  uint32_t* bail = nullptr;      // kBailLists lists of cap lanes each, then the wave lists (bail_words)
  uint64_t* tick_stage = nullptr;  // a TickStage record per tick-list entry (gr_layout.h)
  uint32_t* counters = nullptr;  // [2 (pass parity)][kCounters][kCounterStride]
  // gr_step_device passes of at least this many lanes run the role instances
  // (StepParams::split); GR_SPLIT_MIN_LANES at gr_create overrides it (tests)
  uint32_t split_min = kSplitMinLanes;
  // passes of at most this many workgroups run fused (gr_small_kernel);
  // GR_SMALL_BLOCKS at gr_create overrides it (0: never; tests and A/B runs)
  uint32_t small_blocks = kSmallBlocks;
  uint8_t* hints = nullptr;      // 2 x [hint_stride(cap)] wave hints of the device-resident path (gr_layout.h WH_*):
                                 // one set read by a pass, the other written for the next
  uint64_t hint_flip = 0;
  uint64_t launches = 0;         // never reset: selects the live counter set
  uint64_t timing_bailed0 = 0;   // ST_BAILED when timing began
  bool timing = false;
  std::vector<PassTiming> timings;  // one per pass while timing
  bool routes_bound = false;
  uint8_t route_mode = RT_TABLE;  // of the bound routes (RT_TABLE, RT_AFFINE or RT_LOOPBACK)
  uint32_t route_g = 0, route_r = 0;
  uint32_t* route_base = nullptr;  // device [2][GR_SMAX][GR_SMAX]
  bool locals_set = false;
  bool locals_other = false;  // some bound local input has ticks / a ReadIndex / oversized counts (LW_OTHER)
  uint64_t passes = 0;
  // GR_WAVE_CLOCK=<path> at gr_create (profiling): the general kernel records
  // each wave's span; gr_destroy writes the last pass's records to <path>
  uint64_t* wclock = nullptr;
  uint8_t bin_general = 1;  // StepParams::bin_general (GR_BIN_GENERAL=0 at gr_create: off, A/B runs)
  uint32_t* tail_hint = nullptr;  // StepParams::tail_hint: pinned, host-visible (GR_TAIL_HINT=0: off)
  uint8_t tail_mode = 0;          // StepParams::tail_mode (GR_TAIL_MODE at gr_create: tests, A/B runs)
  std::string wclock_path;

  // gr_step buffers (gr_io.h), grown on demand and reused
  struct Buf {
    void* p = nullptr;
    size_t n = 0;
  };
  Buf d_in, d_out;          // mailbox spaces
  Buf d_msgs, d_locals;     // caller records, as given
  Buf d_mark, d_lop;        // [max_peers] input flags, lane of peer
  Buf d_keys, d_idx, d_skeys, d_sidx;  // mailbox sort
  Buf d_win, d_oc, d_off;   // [lanes]
  Buf d_tmp;                // scan tile sums (io_scan)
  Buf d_kcnt, d_kbase;      // sort_keys: records per mailbox and their exclusive scan
  Buf d_scal;               // lane count, error, outbox total
  Buf d_outmsgs, d_results; // packed outbox
  Buf d_peers, d_slots;     // gr_peer records of a load/sync, slot list
  Buf d_ext, d_lext;        // gr_step_compact: ext message / local records
  Buf d_oc64, d_off64, d_rx, d_roff;  // compact outbox counts and offsets
  Buf d_outext, d_resext;   // compact outbox ext records
  Buf d_nodes;              // gr_bind_nodes: (cluster, node) -> slot table
  Buf d_wrec, d_why, d_unr; // gr_step_wire: routed records, per-message reason, unrouted indices
  uint32_t nodes_cap = 0;
  uint8_t* h_unr = nullptr;  // pinned: unrouted indices + reasons
  size_t h_unr_bytes = 0;
  uint8_t* h_inmsgs = nullptr;   // pinned inbox the caller may fill in place (gr_inbox_reserve)
  uint8_t* h_inlocals = nullptr;
  size_t h_inmsgs_bytes = 0, h_inlocals_bytes = 0;
  uint8_t* h_outmsgs = nullptr;  // pinned: returned to the caller until gr_release_outbox
  uint8_t* h_results = nullptr;
  uint8_t* h_scal = nullptr;
  size_t h_outmsgs_bytes = 0, h_results_bytes = 0, h_scal_bytes = 0;
  uint8_t* h_inext = nullptr;  // gr_cinbox_reserve's ext arrays (the compact ones reuse h_inmsgs / h_inlocals)
  uint8_t* h_inlext = nullptr;
  size_t h_inext_bytes = 0, h_inlext_bytes = 0;
  uint8_t* h_outext = nullptr;  // gr_step_compact's ext outputs (the compact ones reuse h_outmsgs / h_results)
  uint8_t* h_resext = nullptr;
  size_t h_outext_bytes = 0, h_resext_bytes = 0;
  std::mutex mu;  // one host-path pass at a time per engine
  // gr_step_compact_begin -> _end: the uploaded pass waiting for its second half
  struct CPending {
    bool on = false;
    uint32_t nm = 0, nlc = 0, nx = 0, nlx = 0, nl = 0;
  } cpend;
  // cpend.on, readable without the mutex: between _begin and _end the pending
  // pass owns the shared scratch (d_mark, d_lop, d_msgs, d_locals, d_ext,
  // d_lext, d_scal) and the lane rows, so every other entry point that uses
  // them or steps the engine refuses with GR_ESTATE until _end has run.
  std::atomic<bool> pending{false};
};

// GR_ESTATE while a gr_step_compact_begin waits for its _end (gpuraft.h).
#define GR_REFUSE_PENDING(e)                          \
  do {                                                \
    if ((e)->pending.load(std::memory_order_acquire)) \
      return GR_ESTATE;                               \
  } while (0)

// A fresh timing record for the next pass (nullptr when timing is off or a
// HIP call fails: the pass then runs untimed and gr_timing_end reports it).
static PassTiming* next_timing(gr_engine* e) {
  if (!e->timing) return nullptr;
  PassTiming t{};
  for (int k = 0; k < 3; ++k)
    if (hipEventCreate(&t.ev[k]) != hipSuccess) return nullptr;
  e->timings.push_back(t);
  return &e->timings.back();
}

static void free_timings(gr_engine* e) {
  for (auto& t : e->timings) {
    for (int k = 0; k < 3; ++k) (void)hipEventDestroy(t.ev[k]);
  }
  e->timings.clear();
}

namespace {

#ifndef GR_INBOX_WC
#define GR_INBOX_WC 1
#endif
const unsigned kInboxPinned = GR_INBOX_WC ? (hipHostMallocDefault | hipHostMallocWriteCombined) : hipHostMallocDefault;

// GR_PHASES=1: host-side phase times of a boundary pass on stderr (profiling aid).
struct PhaseClock {
  bool on = getenv("GR_PHASES") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  char buf[256];
  int len = 0;
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    len += snprintf(buf + len, sizeof(buf) - len, "%s %.3f ms; ", what,
                    std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
  void report() {
    if (on) fprintf(stderr, "gr_phases: %s\n", buf);
  }
};

#define HIPCHK(x)                              \
  do {                                         \
    hipError_t _e = (x);                       \
    if (_e != hipSuccess) return GR_EDEVICE;   \
  } while (0)

StepParams base_params(gr_engine* e) {
  StepParams kp;
  memset(&kp, 0, sizeof(kp));
  kp.st = e->st;
  kp.ln = e->ln;
  kp.stats = e->stats;
  kp.max_entry_size = e->cfg.max_entry_size;
  kp.small_blocks = e->small_blocks;
  kp.wclock = e->wclock;
  kp.bin_general = e->bin_general;
  kp.tail_hint = e->tail_hint;
  kp.tail_mode = e->tail_mode;
  kp.tick_stage = e->tick_stage;
  return kp;
}

int grow_device(void** p, size_t* have, size_t want) {
  if (*have >= want) return GR_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *have = 0;
  HIPCHK(hipMalloc(p, want));
  *have = want;
  return GR_OK;
}
// flags: hipHostMallocDefault for what the host reads (outboxes), write-combined
// for the inboxes the host only writes and the device reads once (no snooping of
// dirty host cache lines during the upload).
int grow_pinned(uint8_t** p, size_t* have, size_t want, unsigned flags = hipHostMallocDefault) {
  if (*have >= want) return GR_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *have = 0;
  HIPCHK(hipHostMalloc((void**)p, want, flags));
  *have = want;
  return GR_OK;
}

// Grid of a boundary pass (grid-stride loops): enough workgroups to fill the chip.
uint32_t io_grid(size_t n) {
  const size_t b = (n + io::kIoBlock - 1) / io::kIoBlock;
  return (uint32_t)std::max<size_t>(1, std::min<size_t>(b, 4096));
}

// gr_peer records <-> state rows for slots [first, first+n) or a slot list
// (gr_io.h): the records cross PCIe once, the transpose runs on the device.
int transfer(gr_engine* e, const uint32_t* slots, uint32_t first, size_t n, gr_peer* host, bool to_device) {
  if (!e || (n && !host)) return GR_EINVAL;
  const uint32_t cap = e->cfg.max_peers;
  if (!slots && (uint64_t)first + n > cap) return GR_ERANGE;
  if (n == 0) return GR_OK;
  if (n >= 0x80000000ull) return GR_EINVAL;
  if (slots && !to_device)
    for (size_t x = 0; x < n; ++x)
      if (slots[x] >= cap) return GR_ERANGE;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  HIPCHK(hipDeviceSynchronize());  // passes in flight on other streams own the rows
  const hipStream_t s = e->stream;
  const size_t bytes = n * sizeof(gr_peer);
  int r;
  if ((r = grow_device(&e->d_peers.p, &e->d_peers.n, bytes))) return r;
  const uint32_t* dslots = nullptr;
  if (slots) {
    if ((r = grow_device(&e->d_slots.p, &e->d_slots.n, n * 4))) return r;
    HIPCHK(hipMemcpyAsync(e->d_slots.p, slots, n * 4, hipMemcpyHostToDevice, s));
    dslots = (const uint32_t*)e->d_slots.p;
  }
  gr_peer* dp = (gr_peer*)e->d_peers.p;
  const dim3 grid(io_grid(n)), blk(io::kIoBlock);
  if (to_device) {
    if ((r = grow_device(&e->d_mark.p, &e->d_mark.n, (size_t)cap * 4))) return r;
    if ((r = grow_device(&e->d_scal.p, &e->d_scal.n, 16))) return r;
    if ((r = grow_pinned(&e->h_scal, &e->h_scal_bytes, 16))) return r;
    HIPCHK(hipMemcpyAsync(dp, host, bytes, hipMemcpyHostToDevice, s));
    if (slots) HIPCHK(hipMemsetAsync(e->d_mark.p, 0, (size_t)cap * 4, s));
    HIPCHK(hipMemsetAsync(e->d_scal.p, 0, 16, s));
    hipLaunchKernelGGL(io::check_peers, grid, blk, 0, s, (const gr_peer*)dp, dslots, (uint32_t)n, e->S, cap,
                       (uint32_t*)e->d_mark.p, (uint32_t*)e->d_scal.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(e->h_scal, e->d_scal.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const uint32_t err = *(uint32_t*)e->h_scal;
    if (err & io::ERR_SLOT) return GR_ERANGE;  // no row was written
    if (err & io::ERR_PEER) return GR_EINVAL;
    hipLaunchKernelGGL(io::peers_to_rows, grid, blk, 0, s, (const gr_peer*)dp, dslots, first, (uint32_t)n, e->st,
                       e->S);
    HIPCHK(hipGetLastError());
  } else {
    HIPCHK(hipMemsetAsync(dp, 0, bytes, s));
    hipLaunchKernelGGL(io::rows_to_peers, grid, blk, 0, s, e->st, dslots, first, (uint32_t)n, e->S, dp);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(host, dp, bytes, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  return GR_OK;
}

// Exclusive sum of n values on `s` (gr_scan.h), the tile sums in e->d_tmp.
template <class T>
int io_scan_t(gr_engine* e, const T* in, T* out, uint32_t n, hipStream_t s) {
  if (n == 0) return GR_OK;
  const int r = grow_device(&e->d_tmp.p, &e->d_tmp.n, (size_t)scan::scan_tiles_of(n) * sizeof(T));
  if (r) return r;
  HIPCHK(scan::exclusive_scan<T>(in, out, n, (T*)e->d_tmp.p, s));
  return GR_OK;
}
int io_scan(gr_engine* e, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s) {
  return io_scan_t<uint32_t>(e, in, out, n, s);
}
int io_scan64(gr_engine* e, const uint64_t* in, uint64_t* out, uint32_t n, hipStream_t s) {
  return io_scan_t<uint64_t>(e, in, out, n, s);
}

// Stable sort of the inbox's mailbox keys (slot-major j*nl + lane, each below
// `positions`), so arrival order inside a mailbox survives: a counting sort
// (gr_io.h key_count, key_scatter, key_order); sorted keys/indexes in
// d_skeys/d_sidx. d_idx holds each record's slot in its mailbox meanwhile.
int sort_keys(gr_engine* e, uint32_t nm, uint32_t positions, hipStream_t s) {
  int r;
  if ((r = grow_device(&e->d_kcnt.p, &e->d_kcnt.n, (size_t)positions * 4 + 4))) return r;
  if ((r = grow_device(&e->d_kbase.p, &e->d_kbase.n, (size_t)positions * 4 + 4))) return r;
  uint32_t* cnt = (uint32_t*)e->d_kcnt.p;
  uint32_t* base = (uint32_t*)e->d_kbase.p;
  HIPCHK(hipMemsetAsync(cnt, 0, (size_t)positions * 4, s));
  const dim3 blk(io::kIoBlock);
  hipLaunchKernelGGL(io::key_count, dim3(io_grid(nm)), blk, 0, s, (const uint32_t*)e->d_keys.p, nm, cnt,
                     (uint32_t*)e->d_idx.p);
  HIPCHK(hipGetLastError());
  if ((r = io_scan(e, cnt, base, positions, s))) return r;
  hipLaunchKernelGGL(io::key_scatter, dim3(io_grid(nm)), blk, 0, s, (const uint32_t*)e->d_keys.p,
                     (const uint32_t*)e->d_idx.p, nm, (const uint32_t*)base, (uint32_t*)e->d_skeys.p,
                     (uint32_t*)e->d_sidx.p);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(io::key_order, dim3(io_grid(positions)), blk, 0, s, (const uint32_t*)cnt,
                     (const uint32_t*)base, positions, (uint32_t*)e->d_sidx.p);
  HIPCHK(hipGetLastError());
  return GR_OK;
}

}  // namespace

extern "C" {

const char* gr_strerror(int err) {
  switch (err) {
    case GR_OK: return "ok";
    case GR_EINVAL: return "invalid argument";
    case GR_ENOMEM: return "out of memory";
    case GR_EDEVICE: return "HIP device error";
    case GR_ERANGE: return "slot range out of bounds";
    case GR_ECAPACITY: return "mailbox capacity exceeded";
    case GR_ESTATE: return "engine state error";
  }
  return "unknown error";
}

const char* gr_escalation_name(int esc) {
  static const char* names[] = {"none", "term_window", "random", "unsupported", "election", "panic",
                                "capacity", "snapshot", "entry_size", "msg_runs", "nonmember",
                                "config_change", "wide_term"};
  if (esc < 0 || esc > GR_ESC_WIDE_TERM) return "unknown";
  return names[esc];
}

int gr_create(const gr_config* cfg, gr_engine** out) {
  if (!cfg || !out) return GR_EINVAL;
  *out = nullptr;
  if (cfg->window_runs != GR_K || cfg->read_index_depth != GR_Q || cfg->mailbox_depth != GR_C)
    return GR_EINVAL;
  if (cfg->max_peers == 0 || cfg->slots == 0 || cfg->slots > GR_SMAX) return GR_EINVAL;
  const uint32_t S = instantiated_slots(cfg->slots);
  if (!S) return GR_EINVAL;
  if (hipSetDevice((int)cfg->device) != hipSuccess) return GR_EDEVICE;
  gr_engine* e = new (std::nothrow) gr_engine();
  if (!e) return GR_ENOMEM;
  e->cfg = *cfg;
  e->S = S;
  e->cap = pad_cap(cfg->max_peers);
  e->st.cap = e->cap;
  e->st.S = S;
  e->ln.lcap = e->cap;
  e->ln.S = S;
  const size_t sb = state_bytes(S, e->cap), lb = lane_bytes(S, e->cap);
  e->stats_rows = (e->cap + kBlock - 1) / kBlock;
  if (const char* sm = getenv("GR_SPLIT_MIN_LANES")) {
    const long v = strtol(sm, nullptr, 10);
    if (v > 0) e->split_min = (uint32_t)v;
  }
  if (const char* sb = getenv("GR_SMALL_BLOCKS")) e->small_blocks = (uint32_t)strtoul(sb, nullptr, 10);
  if (const char* bg = getenv("GR_BIN_GENERAL")) e->bin_general = bg[0] == '1';
  if (const char* tm = getenv("GR_TAIL_MODE")) e->tail_mode = (uint8_t)(strtoul(tm, nullptr, 10) & 3u);
  if (const char* wc = getenv("GR_WAVE_CLOCK")) {
    // two regions: the general kernel's waves, then the tick kernel's (gr_kernels.h)
    if (hipMalloc((void**)&e->wclock, 2 * (size_t)kGeneralWaveSlots * kWaveClockWords * 8) == hipSuccess &&
        hipMemset(e->wclock, 0, 2 * (size_t)kGeneralWaveSlots * kWaveClockWords * 8) == hipSuccess)
      e->wclock_path = wc;
  }
  void *ds = nullptr, *dl = nullptr;
  if (hipMalloc(&ds, sb) != hipSuccess || hipMalloc(&dl, lb) != hipSuccess ||
      hipMalloc((void**)&e->stats, (size_t)e->stats_rows * NSTAT * 8) != hipSuccess ||
      hipMalloc((void**)&e->bail, bail_words(e->cap) * 4) != hipSuccess ||
      hipMalloc((void**)&e->tick_stage, (size_t)kTickLists * tick_cap(e->cap) * kTickStageWords * 8) != hipSuccess ||
      hipMalloc((void**)&e->counters, 2 * kCounters * kCounterStride * 4) != hipSuccess ||
      hipMalloc((void**)&e->route_base, 2 * GR_SMAX * GR_SMAX * 4) != hipSuccess ||
      hipMalloc((void**)&e->hints, 2 * hint_stride(e->cap)) != hipSuccess) {
    if (ds) (void)hipFree(ds);
    if (dl) (void)hipFree(dl);
    e->st.base = nullptr;
    e->ln.base = nullptr;
    gr_destroy(e);
    return GR_ENOMEM;
  }
  e->st.base = (uint8_t*)ds;
  e->ln.base = (uint8_t*)dl;
  if (hipMemset(ds, 0, sb) != hipSuccess || hipMemset(dl, 0, lb) != hipSuccess ||
      hipMemset(e->stats, 0, (size_t)e->stats_rows * NSTAT * 8) != hipSuccess ||
      hipMemset(e->counters, 0, 2 * kCounters * kCounterStride * 4) != hipSuccess ||
      hipMemset(e->hints, 0, 2 * hint_stride(e->cap)) != hipSuccess ||
      hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    gr_destroy(e);
    return GR_EDEVICE;
  }
  const char* th = getenv("GR_TAIL_HINT");
  if (!(th && th[0] == '0')) {  // a failed allocation only leaves the grids full
    if (hipHostMalloc((void**)&e->tail_hint, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
      e->tail_hint = nullptr;
    else
      *(volatile uint32_t*)e->tail_hint = kTailAll;
  }
  *out = e;
  return GR_OK;
}

void gr_destroy(gr_engine* e) {
  if (!e) return;
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->st.base) (void)hipFree(e->st.base);
  if (e->ln.base) (void)hipFree(e->ln.base);
  if (e->stats) (void)hipFree(e->stats);
  if (e->bail) (void)hipFree(e->bail);
  if (e->tick_stage) (void)hipFree(e->tick_stage);
  if (e->counters) (void)hipFree(e->counters);
  if (e->route_base) (void)hipFree(e->route_base);
  if (e->hints) (void)hipFree(e->hints);
  if (e->tail_hint) (void)hipHostFree(e->tail_hint);
  if (e->wclock) {
    std::vector<uint64_t> h(2 * (size_t)kGeneralWaveSlots * kWaveClockWords);
    if (!e->wclock_path.empty() && hipStreamSynchronize(e->stream) == hipSuccess &&
        hipMemcpy(h.data(), e->wclock, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      if (FILE* f = fopen(e->wclock_path.c_str(), "wb")) {
        fwrite(h.data(), 8, h.size(), f);
        fclose(f);
      }
    }
    (void)hipFree(e->wclock);
  }
  free_timings(e);
  for (gr_engine::Buf* b : {&e->d_in, &e->d_out, &e->d_msgs, &e->d_locals, &e->d_mark, &e->d_lop, &e->d_keys,
                            &e->d_idx, &e->d_skeys, &e->d_sidx, &e->d_win, &e->d_oc, &e->d_off, &e->d_tmp,
                            &e->d_scal, &e->d_outmsgs, &e->d_results, &e->d_peers, &e->d_slots, &e->d_ext,
                            &e->d_lext, &e->d_oc64, &e->d_off64, &e->d_rx, &e->d_roff, &e->d_outext,
                            &e->d_resext, &e->d_nodes, &e->d_wrec, &e->d_why, &e->d_unr, &e->d_kcnt, &e->d_kbase})
    if (b->p) (void)hipFree(b->p);
  for (uint8_t* h : {e->h_outmsgs, e->h_results, e->h_scal, e->h_inmsgs, e->h_inlocals, e->h_inext, e->h_inlext,
                     e->h_outext, e->h_resext, e->h_unr})
    if (h) (void)hipHostFree(h);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

int gr_load_groups(gr_engine* e, uint32_t first, const gr_peer* peers, size_t n) {
  return transfer(e, nullptr, first, n, const_cast<gr_peer*>(peers), true);
}

int gr_sync_groups_to_host(gr_engine* e, uint32_t first, gr_peer* out, size_t n) {
  return transfer(e, nullptr, first, n, out, false);
}

int gr_load_peers(gr_engine* e, const uint32_t* slots, const gr_peer* peers, size_t n) {
  if (n && !slots) return GR_EINVAL;
  return transfer(e, slots, 0, n, const_cast<gr_peer*>(peers), true);
}

int gr_sync_peers_to_host(gr_engine* e, const uint32_t* slots, gr_peer* out, size_t n) {
  if (n && !slots) return GR_EINVAL;
  return transfer(e, slots, 0, n, out, false);
}

// LogReader.Compact(index) (logreader.go:251-269) for a slot list, mirrored
// into the device's firstIndex-1 (entryLog.firstIndex, logentry.go:97-104):
// after compaction term() answers 0 below it and Replicate sends below it take
// the snapshot path, as in the reference.
int gr_compact_log(gr_engine* e, const uint32_t* slots, const uint64_t* index, size_t n, int32_t* status) {
  if (!e || (n && (!slots || !index))) return GR_EINVAL;
  if (n == 0) return GR_OK;
  if (n >= 0x80000000ull) return GR_EINVAL;
  const uint32_t cap = e->cfg.max_peers;
  std::vector<uint64_t> seen((cap + 63) / 64, 0);
  for (size_t x = 0; x < n; ++x) {
    const uint32_t p = slots[x];
    if (p >= cap || (seen[p >> 6] >> (p & 63)) & 1) return GR_ERANGE;  // nothing written
    seen[p >> 6] |= 1ull << (p & 63);
  }
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  HIPCHK(hipDeviceSynchronize());  // passes in flight on other streams own the rows
  const hipStream_t s = e->stream;
  int r;
  if ((r = grow_device(&e->d_slots.p, &e->d_slots.n, n * 4))) return r;
  if ((r = grow_device(&e->d_peers.p, &e->d_peers.n, n * 12 + 16))) return r;
  if ((r = grow_device(&e->d_scal.p, &e->d_scal.n, 16))) return r;
  if ((r = grow_pinned(&e->h_scal, &e->h_scal_bytes, 16))) return r;
  uint64_t* didx = (uint64_t*)e->d_peers.p;
  int32_t* dst = (int32_t*)(didx + n);
  HIPCHK(hipMemcpyAsync(e->d_slots.p, slots, n * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(didx, index, n * 8, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(e->d_scal.p, 0, 16, s));
  const dim3 grid(io_grid(n)), blk(io::kIoBlock);
  const uint32_t* ds = (const uint32_t*)e->d_slots.p;
  uint32_t* refused = (uint32_t*)e->d_scal.p;
  switch (e->S) {
#define GR_COMPACT_CASE(SS)                                                                                 \
  case SS:                                                                                                  \
    hipLaunchKernelGGL(io::compact_rows<SS>, grid, blk, 0, s, e->st, ds, (const uint64_t*)didx, (uint32_t)n, \
                       dst, refused);                                                                       \
    break;
    GR_COMPACT_CASE(1) GR_COMPACT_CASE(2) GR_COMPACT_CASE(3) GR_COMPACT_CASE(4)
    GR_COMPACT_CASE(5) GR_COMPACT_CASE(6) GR_COMPACT_CASE(7) GR_COMPACT_CASE(8)
#undef GR_COMPACT_CASE
    default: return GR_EINVAL;
  }
  HIPCHK(hipGetLastError());
  if (status) HIPCHK(hipMemcpyAsync(status, dst, n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(e->h_scal, refused, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return *(uint32_t*)e->h_scal ? GR_ESTATE : GR_OK;
}

// entryLog.commitUpdate (logentry.go:325-335) for a slot list: the host's
// persistence/apply acknowledgement moves inMemory.savedTo / markerIndex and
// entryLog.applied on the device (gr_io.h commit_rows).
int gr_commit_update(gr_engine* e, const uint32_t* slots, const gr_update_commit* uc, size_t n, int32_t* status) {
  if (!e || (n && (!slots || !uc))) return GR_EINVAL;
  if (n == 0) return GR_OK;
  if (n >= 0x80000000ull) return GR_EINVAL;
  const uint32_t cap = e->cfg.max_peers;
  std::vector<uint64_t> seen((cap + 63) / 64, 0);
  for (size_t x = 0; x < n; ++x) {
    const uint32_t p = slots[x];
    if (p >= cap || (seen[p >> 6] >> (p & 63)) & 1) return GR_ERANGE;  // nothing written
    seen[p >> 6] |= 1ull << (p & 63);
  }
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  HIPCHK(hipDeviceSynchronize());  // passes in flight on other streams own the rows
  const hipStream_t s = e->stream;
  int r;
  if ((r = grow_device(&e->d_slots.p, &e->d_slots.n, n * 4))) return r;
  if ((r = grow_device(&e->d_peers.p, &e->d_peers.n, n * (sizeof(gr_update_commit) + 4) + 16))) return r;
  if ((r = grow_device(&e->d_scal.p, &e->d_scal.n, 16))) return r;
  if ((r = grow_pinned(&e->h_scal, &e->h_scal_bytes, 16))) return r;
  gr_update_commit* duc = (gr_update_commit*)e->d_peers.p;
  int32_t* dst = (int32_t*)(duc + n);
  HIPCHK(hipMemcpyAsync(e->d_slots.p, slots, n * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(duc, uc, n * sizeof(gr_update_commit), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(e->d_scal.p, 0, 16, s));
  const dim3 grid(io_grid(n)), blk(io::kIoBlock);
  const uint32_t* ds = (const uint32_t*)e->d_slots.p;
  uint32_t* refused = (uint32_t*)e->d_scal.p;
  hipLaunchKernelGGL(io::commit_rows, grid, blk, 0, s, e->st, ds, (const gr_update_commit*)duc, (uint32_t)n, dst,
                     refused);
  HIPCHK(hipGetLastError());
  if (status) HIPCHK(hipMemcpyAsync(status, dst, n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(e->h_scal, refused, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return *(uint32_t*)e->h_scal ? GR_ESTATE : GR_OK;
}

// Peer.NotifyRaftLastApplied (peer.go:282-284) for a slot list: raft.applied =
// the RSM's batched last applied index, as node.handleEvents does first in
// every step (node.go:632-635,653). No other field changes.
int gr_notify_applied(gr_engine* e, const uint32_t* slots, const uint64_t* applied, size_t n) {
  if (!e || (n && (!slots || !applied))) return GR_EINVAL;
  if (n == 0) return GR_OK;
  if (n >= 0x80000000ull) return GR_EINVAL;
  const uint32_t cap = e->cfg.max_peers;
  std::vector<uint64_t> seen((cap + 63) / 64, 0);
  for (size_t x = 0; x < n; ++x) {
    const uint32_t p = slots[x];
    if (p >= cap || (seen[p >> 6] >> (p & 63)) & 1) return GR_ERANGE;  // nothing written
    seen[p >> 6] |= 1ull << (p & 63);
  }
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  HIPCHK(hipDeviceSynchronize());  // passes in flight on other streams own the rows
  const hipStream_t s = e->stream;
  int r;
  if ((r = grow_device(&e->d_slots.p, &e->d_slots.n, n * 4))) return r;
  if ((r = grow_device(&e->d_peers.p, &e->d_peers.n, n * 8))) return r;
  HIPCHK(hipMemcpyAsync(e->d_slots.p, slots, n * 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(e->d_peers.p, applied, n * 8, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(io::set_row_u64, dim3(io_grid(n)), dim3(io::kIoBlock), 0, s, e->st, (uint32_t)SR_APPLIED,
                     (const uint32_t*)e->d_slots.p, (const uint64_t*)e->d_peers.p, (uint32_t)n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  return GR_OK;
}

uint64_t gr_space_chunk_bytes(uint32_t positions, uint32_t depth) {
  if (depth == 0 || depth > GR_C) return 0;
  return space_chunk_bytes_pc(space_pad_positions(positions), depth);
}
uint64_t gr_space_bytes(uint32_t n_chunks, uint32_t positions, uint32_t depth) {
  return (uint64_t)n_chunks * gr_space_chunk_bytes(positions, depth);
}
uint64_t gr_space_hot_chunk_bytes(uint32_t positions, uint32_t depth) {
  if (depth == 0 || depth > GR_C) return 0;
  return space_hot_chunk_bytes_pc(space_pad_positions(positions), depth);
}
uint32_t gr_space_tile_positions(void) { return kTileW; }
uint64_t gr_space_hot_tile_bytes(uint32_t depth) {
  if (depth == 0 || depth > GR_C) return 0;
  return tile_hot_bytes(depth);
}

int gr_space_cold_used(gr_engine* e, const void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                       void* stream, uint32_t* out) {
  if (!e || !space || !out || depth == 0 || depth > GR_C) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  int r;
  if ((r = grow_device(&e->d_scal.p, &e->d_scal.n, 16))) return r;
  if ((r = grow_pinned(&e->h_scal, &e->h_scal_bytes, 16))) return r;
  const hipStream_t s = (hipStream_t)stream;
  const SpaceView v = make_view(space, n_chunks, positions, depth);
  uint32_t* flag = (uint32_t*)e->d_scal.p + 3;
  HIPCHK(hipMemsetAsync(flag, 0, 4, s));
  hipLaunchKernelGGL(io::cold_used, dim3(io_grid((size_t)n_chunks * v.pc)), dim3(io::kIoBlock), 0, s, v, flag);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_scal + 12, flag, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *out = *(uint32_t*)(e->h_scal + 12);
  return GR_OK;
}

uint64_t gr_space_side_bytes(uint32_t n_chunks, uint32_t depth, uint32_t capacity) {
  if (depth == 0 || depth > GR_C) return 0;
  return (uint64_t)n_chunks * io::side_chunk_bytes(depth, capacity);
}

int gr_space_side_pack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, void* side,
                       uint32_t capacity, void* stream) {
  if (!space || !side || depth == 0 || depth > GR_C || n_chunks == 0) return GR_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  const SpaceView v = make_view(space, n_chunks, positions, depth);
  for (uint32_t c = 0; c < n_chunks; ++c)
    HIPCHK(hipMemsetAsync((uint8_t*)side + (uint64_t)c * io::side_chunk_bytes(depth, capacity), 0, io::kSideHdr, s));
  hipLaunchKernelGGL(io::side_pack, dim3(io_grid((size_t)n_chunks * v.pc)), dim3(io::kIoBlock), 0, s, v,
                     (uint8_t*)side, capacity);
  HIPCHK(hipGetLastError());
  return GR_OK;
}

int gr_space_side_unpack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, const void* side,
                         uint32_t capacity, void* stream) {
  if (!space || !side || depth == 0 || depth > GR_C || n_chunks == 0) return GR_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  const SpaceView v = make_view(space, n_chunks, positions, depth);
  if (capacity) {
    hipLaunchKernelGGL(io::side_unpack, dim3(io_grid((size_t)n_chunks * capacity)), dim3(io::kIoBlock), 0, s, v,
                       (const uint8_t*)side, capacity);
    HIPCHK(hipGetLastError());
  }
  return GR_OK;
}

int gr_space_side_pack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                            void* side_host, uint32_t capacity) {
  if (!space_host || !side_host || depth == 0 || depth > GR_C || n_chunks == 0) return GR_EINVAL;
  const SpaceView v = make_view(space_host, n_chunks, positions, depth);
  uint8_t* side = (uint8_t*)side_host;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    uint32_t* cnt = (uint32_t*)(side + (uint64_t)c * io::side_chunk_bytes(depth, capacity));
    *cnt = 0;
    for (uint32_t l = 0; l < v.pc; ++l) {
      const uint32_t g = c * v.pc + l;
      if (io::needs_cold(v.at(g).cnt())) io::side_put(v, g, side, capacity, (*cnt)++);
    }
  }
  return GR_OK;
}

int gr_space_side_unpack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                              const void* side_host, uint32_t capacity) {
  if (!space_host || !side_host || depth == 0 || depth > GR_C || n_chunks == 0) return GR_EINVAL;
  const SpaceView v = make_view(space_host, n_chunks, positions, depth);
  const uint8_t* side = (const uint8_t*)side_host;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    const uint8_t* h = side + (uint64_t)c * io::side_chunk_bytes(depth, capacity);
    const uint32_t n = *(const uint32_t*)h;
    for (uint32_t x = 0; x < n && x < capacity; ++x) {
      const uint8_t* e = h + io::kSideHdr + (uint64_t)x * io::side_entry_bytes(depth);
      io::cold_scatter(v.at(c * v.pc + ((const uint32_t*)e)[0]), mb_n(((const uint32_t*)e)[1]), e);
    }
  }
  return GR_OK;
}

uint64_t gr_space_cx_bytes(uint32_t n_chunks, uint32_t positions, uint32_t depth, const uint32_t* capacities,
                           uint32_t side_capacity) {
  if (depth == 0 || depth > GR_C || !capacities || n_chunks > io::kCxMaxChunks) return 0;
  return io::cx_caps(space_pad_positions(positions), depth, n_chunks, capacities, side_capacity).off[n_chunks];
}

#define GR_CX_ARGS_OK(space, cx, depth, n_chunks, capacities)                                                  \
  ((space) && (cx) && (capacities) && (depth) > 0 && (depth) <= GR_C && (n_chunks) > 0 &&                     \
   (n_chunks) <= io::kCxMaxChunks)

int gr_space_cx_pack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, void* cx,
                     const uint32_t* capacities, uint32_t side_capacity, void* stream) {
  if (!GR_CX_ARGS_OK(space, cx, depth, n_chunks, capacities)) return GR_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  const SpaceView v = make_view(space, n_chunks, positions, depth);
  const io::CxCaps C = io::cx_caps(v.pc, depth, n_chunks, capacities, side_capacity);
  for (uint32_t c = 0; c < n_chunks; ++c) HIPCHK(hipMemsetAsync((uint8_t*)cx + C.off[c], 0, io::kCxHdr, s));
  const uint32_t nwv = v.pc / 64;
  hipLaunchKernelGGL(io::cx_pack, dim3((nwv + io::kCxPackGroups - 1) / io::kCxPackGroups, n_chunks),
                     dim3(io::kIoBlock), 0, s, v, (uint8_t*)cx, C);
  HIPCHK(hipGetLastError());
  return GR_OK;
}

int gr_space_cx_unpack(void* space, uint32_t n_chunks, uint32_t positions, uint32_t depth, const void* cx,
                       const uint32_t* capacities, uint32_t side_capacity, void* stream) {
  if (!GR_CX_ARGS_OK(space, cx, depth, n_chunks, capacities)) return GR_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  const SpaceView v = make_view(space, n_chunks, positions, depth);
  const io::CxCaps C = io::cx_caps(v.pc, depth, n_chunks, capacities, side_capacity);
  const uint32_t nwv = v.pc / 64;
  hipLaunchKernelGGL(io::cx_unpack_waves, dim3((nwv + io::kCxUnpackGroups - 1) / io::kCxUnpackGroups, n_chunks),
                     dim3(io::kIoBlock), 0, s, v, (const uint8_t*)cx, C);
  HIPCHK(hipGetLastError());
  if (side_capacity) {
    hipLaunchKernelGGL(io::cx_unpack_side, dim3(io_grid((size_t)n_chunks * side_capacity)), dim3(io::kIoBlock), 0, s,
                       v, (const uint8_t*)cx, C);
    HIPCHK(hipGetLastError());
  }
  return GR_OK;
}

// The same codec over host memory (tests): records in the device's regions
// (wave group wl belongs to pack workgroup wl / kCxPackGroups, whose region is
// that workgroup's index modulo cx_regions), each region and the side entries
// filled in position order (the device packer's order within a region may
// differ; what unpacks does not).
int gr_space_cx_pack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth, void* cx_host,
                          const uint32_t* capacities, uint32_t side_capacity) {
  if (!GR_CX_ARGS_OK(space_host, cx_host, depth, n_chunks, capacities)) return GR_EINVAL;
  const SpaceView v = make_view(space_host, n_chunks, positions, depth);
  const io::CxCaps C = io::cx_caps(v.pc, depth, n_chunks, capacities, side_capacity);
  for (uint32_t c = 0; c < n_chunks; ++c) {
    const uint32_t capacity = C.cap[c];
    const io::CxLayout L = io::cx_layout(v.pc, depth, capacity, side_capacity);
    uint8_t* buf = (uint8_t*)cx_host + C.off[c];
    memset(buf, 0, io::kCxHdr);
    uint32_t* ctr = (uint32_t*)buf;
    uint32_t* nside = ctr + io::kCxSub * io::kCxCtr;
    const uint32_t nreg = io::cx_regions(L.nwv);
    for (uint32_t wl = 0; wl < L.nwv; ++wl) {
      const uint32_t reg = (wl / io::kCxPackGroups) % nreg;
      uint32_t roff, rcap;
      io::cx_region(L.nwv, capacity, reg, &roff, &rcap);
      uint32_t* nrec = ctr + reg * io::kCxCtr;
      uint32_t hi = 0;
      bool have = false;
      for (uint32_t lane = 0; lane < 64 && !have; ++lane) {
        const Mailbox mb = v.at(c * v.pc + wl * 64 + lane);
        const uint32_t cb = mb.cnt();
        uint32_t w3;
        uint64_t li;
        bool anch;
        if (mb_n(cb) && io::cx_classify(mb, cb, depth, &w3, &li, &anch) && anch) {
          hi = (uint32_t)(li >> 32);
          have = true;
        }
      }
      uint64_t mask = 0, lost = 0;
      const uint32_t base = roff + *nrec;
      for (uint32_t lane = 0; lane < 64; ++lane) {
        const uint32_t pos = wl * 64 + lane;
        const Mailbox mb = v.at(c * v.pc + pos);
        const uint32_t cb = mb.cnt();
        uint32_t w3 = 0;
        uint64_t li = 0;
        bool anch = false;
        const bool rec = mb_n(cb) && io::cx_classify(mb, cb, depth, &w3, &li, &anch) &&
                         (!anch || (uint32_t)(li >> 32) == hi);
        if (rec && *nrec < rcap) {
          io::cx_put_record(io::cx_term_of(mb, cb), li, w3, buf, L, roff + (*nrec)++);
          mask |= 1ull << lane;
          continue;
        }
        if (rec) ++*nrec;  // counted, as the device's atomic counts it
        if (!mb_n(cb)) continue;
        if (*nside < side_capacity) io::cx_put_side(mb, cb, pos, buf, L, depth, *nside);
        else lost |= 1ull << lane;
        ++*nside;
      }
      uint8_t* h = buf + L.waves + (uint64_t)wl * io::kCxWave;
      ((uint64_t*)h)[0] = mask;
      ((uint64_t*)h)[1] = lost;
      ((uint32_t*)h)[4] = base;
      ((uint32_t*)h)[5] = hi;
    }
  }
  return GR_OK;
}

int gr_space_cx_unpack_host(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                            const void* cx_host, const uint32_t* capacities, uint32_t side_capacity) {
  if (!GR_CX_ARGS_OK(space_host, cx_host, depth, n_chunks, capacities)) return GR_EINVAL;
  const SpaceView v = make_view(space_host, n_chunks, positions, depth);
  const io::CxCaps C = io::cx_caps(v.pc, depth, n_chunks, capacities, side_capacity);
  for (uint32_t c = 0; c < n_chunks; ++c) {
    const io::CxLayout L = io::cx_layout(v.pc, depth, C.cap[c], side_capacity);
    const uint8_t* buf = (const uint8_t*)cx_host + C.off[c];
    for (uint32_t wl = 0; wl < L.nwv; ++wl) {
      const uint8_t* h = buf + L.waves + (uint64_t)wl * io::kCxWave;
      for (uint32_t lane = 0; lane < 64; ++lane)
        io::cx_get_lane(v.at(c * v.pc + wl * 64 + lane), buf, L, ((const uint64_t*)h)[0], ((const uint64_t*)h)[1],
                        ((const uint32_t*)h)[4], ((const uint32_t*)h)[5], lane);
    }
    const uint32_t ns = ((const uint32_t*)buf)[io::kCxSub * io::kCxCtr];
    for (uint32_t x = 0; x < ns && x < side_capacity; ++x) {
      const uint8_t* e = buf + L.side + (uint64_t)x * io::cx_side_entry_bytes(depth);
      io::cx_get_side(v.at(c * v.pc + ((const uint32_t*)e)[0]), e, depth);
    }
  }
  return GR_OK;
}

int gr_space_encode(void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                    const gr_message* msgs, size_t n, const uint32_t* pos_of_msg) {
  if (!space_host || (n && (!msgs || !pos_of_msg)) || depth == 0 || depth > GR_C) return GR_EINVAL;
  const SpaceView v = make_view(space_host, n_chunks, positions, depth);
  for (size_t k = 0; k < n; ++k) {
    const uint32_t g = pos_of_msg[k];
    if (g / v.pc >= n_chunks || g % v.pc >= positions) return GR_ERANGE;
    const Mailbox mb = v.at(g);
    const uint8_t c = (uint8_t)mb_n(mb.cnt());
    if (c >= depth) return GR_ECAPACITY;
    encode_msg(mb, c, msgs[k]);
    mb.cnt() = (uint8_t)(c + 1);
  }
  return GR_OK;
}

int gr_space_decode(const void* space_host, uint32_t n_chunks, uint32_t positions, uint32_t depth,
                    gr_message* out, size_t cap, size_t* n_out) {
  if (!space_host || !n_out || depth == 0 || depth > GR_C) return GR_EINVAL;
  const SpaceView v = make_view(space_host, n_chunks, positions, depth);
  size_t n = 0;
  for (uint32_t c = 0; c < n_chunks; ++c) {
    for (uint32_t l = 0; l < positions; ++l) {
      const uint32_t g = c * v.pc + l;
      const Mailbox mb = v.at(g);
      const uint32_t cb = mb.cnt(), cnt = std::min<uint32_t>(mb_n(cb), depth);
      const bool lost = !(cb & MB_UNIFORM) && (cb & MB_COLD_LOST);  // cold fields not delivered
      for (uint32_t k = 0; k < cnt; ++k) {
        if (out && n < cap) {
          if (lost) {
            memset(&out[n], 0, sizeof(gr_message));
            out[n].reject = 0xFF;  // a record whose fields were lost in the exchange
          } else {
            out[n] = decode_msg(mb, k);
          }
          out[n].peer = g;
          out[n].slot = (uint8_t)k;
        }
        n++;
      }
    }
  }
  *n_out = n;
  return n <= cap || !out ? GR_OK : GR_ECAPACITY;
}

// The device pass of gr_step over nm gr_message records already in e->d_msgs
// (copied from the host by gr_step, or routed from decoded wire records by
// gr_step_wire) and nlc host local inputs. Caller holds e->mu.
static int pack_out_compact(gr_engine* e, uint32_t nl, const SpaceView& vout, gr_coutbox* out, PhaseClock* cl);

// gr_step's device pipeline from inbox records in HBM (e->d_msgs); the outbox as
// full records (out) or, with cout, as compact records (gr_step_wire_compact)
static int step_staged(gr_engine* e, uint32_t nm, const gr_local_input* locals, uint32_t nlc, gr_outbox* out,
                       gr_coutbox* cout = nullptr) {
  if (out) {
    out->msgs = nullptr;
    out->n_msgs = 0;
    out->results = nullptr;
    out->n_results = 0;
  }
  if (cout) memset(cout, 0, sizeof(*cout));
  const uint32_t S = e->S, cap = e->cfg.max_peers;
  if (nm + nlc == 0) return GR_OK;
  const hipStream_t s = e->stream;
  const dim3 blk(io::kIoBlock);
  int r;
  // ---- inbox records -> lanes (gr_io.h)
  if ((r = grow_device(&e->d_locals.p, &e->d_locals.n, (size_t)nlc * sizeof(gr_local_input) + 1))) return r;
  if ((r = grow_device(&e->d_mark.p, &e->d_mark.n, (size_t)cap * 4))) return r;
  if ((r = grow_device(&e->d_lop.p, &e->d_lop.n, (size_t)cap * 4))) return r;
  if ((r = grow_device(&e->d_scal.p, &e->d_scal.n, 16))) return r;
  if ((r = grow_pinned(&e->h_scal, &e->h_scal_bytes, 16))) return r;
  uint32_t* mark = (uint32_t*)e->d_mark.p;
  uint32_t* lop = (uint32_t*)e->d_lop.p;
  uint32_t* scal = (uint32_t*)e->d_scal.p;
  const gr_message* dmsgs = (const gr_message*)e->d_msgs.p;
  const gr_local_input* dloc = (const gr_local_input*)e->d_locals.p;
  if (nlc)
    HIPCHK(hipMemcpyAsync(e->d_locals.p, locals, (size_t)nlc * sizeof(gr_local_input), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(mark, 0, (size_t)cap * 4, s));
  HIPCHK(hipMemsetAsync(scal, 0, 16, s));
  hipLaunchKernelGGL(io::mark_inputs, dim3(io_grid(nm + nlc)), blk, 0, s, dmsgs, nm, dloc, nlc, S, cap, mark,
                     scal + 1);
  HIPCHK(hipGetLastError());
  if ((r = io_scan(e, mark, lop, cap, s))) return r;
  hipLaunchKernelGGL(io::finish_lanes, dim3(1), dim3(64), 0, s, (const uint32_t*)mark, (const uint32_t*)lop, cap,
                     (const uint32_t*)(scal + 1), scal);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_scal, scal, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const uint32_t nl = ((uint32_t*)e->h_scal)[0];
  if (((uint32_t*)e->h_scal)[1]) return GR_EINVAL;  // nothing of the pass ran
  if (nl == 0) return GR_OK;
  uint32_t* peer_of_lane = e->ln.u32(LR_LANE_PEER);
  hipLaunchKernelGGL(io::lane_peers, dim3(io_grid(cap)), blk, 0, s, (const uint32_t*)mark, (const uint32_t*)lop, cap,
                     peer_of_lane);
  HIPCHK(hipGetLastError());
  // ---- mailboxes: slot-major j*nl + lane, arrival order kept by a stable sort
  const uint32_t positions = nl * S;
  const size_t space = gr_space_bytes(1, positions, GR_C);
  if ((r = grow_device(&e->d_in.p, &e->d_in.n, space))) return r;
  if ((r = grow_device(&e->d_out.p, &e->d_out.n, space))) return r;
  const SpaceView vin = make_view(e->d_in.p, 1, positions), vout = make_view(e->d_out.p, 1, positions);
  hipLaunchKernelGGL(io::clear_counts, dim3(io_grid(vin.pc)), blk, 0, s, vin, vin.pc);  // the count bytes
  HIPCHK(hipGetLastError());
  if (nm) {
    for (gr_engine::Buf* b : {&e->d_keys, &e->d_idx, &e->d_skeys, &e->d_sidx})
      if ((r = grow_device(&b->p, &b->n, (size_t)nm * 4))) return r;
    hipLaunchKernelGGL(io::msg_keys, dim3(io_grid(nm)), blk, 0, s, dmsgs, nm, (const uint32_t*)lop, nl,
                       (uint32_t*)e->d_keys.p, (uint32_t*)e->d_idx.p);
    HIPCHK(hipGetLastError());
    if ((r = sort_keys(e, nm, positions, s))) return r;
    hipLaunchKernelGGL(io::encode_sorted, dim3(io_grid(nm)), blk, 0, s, dmsgs, (const uint32_t*)e->d_skeys.p,
                       (const uint32_t*)e->d_sidx.p, nm, vin);
    HIPCHK(hipGetLastError());
  }
  // ---- locals -> lane rows
  if ((r = grow_device(&e->d_win.p, &e->d_win.n, (size_t)nl * 4))) return r;
  HIPCHK(hipMemsetAsync(e->d_win.p, 0, (size_t)nl * 4, s));
  if (nlc) {
    hipLaunchKernelGGL(io::local_winner, dim3(io_grid(nlc)), blk, 0, s, dloc, nlc, (const uint32_t*)lop,
                       (uint32_t*)e->d_win.p);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(io::fill_locals, dim3(io_grid(nl)), blk, 0, s, dloc, (const uint32_t*)e->d_win.p, nl, e->ln);
  HIPCHK(hipGetLastError());
  // ---- the pass
  StepParams kp = base_params(e);
  kp.has_locals = 1;
  kp.has_lane_peer = 1;
  kp.route_mode = RT_IDENTITY;
  kp.in = vin;
  kp.out = vout;
  kp.n_lanes = nl;
  HIPCHK(launch_slots(S, kp, e->bail, e->counters, e->cap, (uint32_t)e->launches++, s, next_timing(e)));
  e->passes++;
  e->locals_set = false;    // the lane rows now hold this pass's compact locals
  e->routes_bound = false;  // and RT_IDENTITY replaced the bound routes
  if (cout) {
    PhaseClock clk;
    return pack_out_compact(e, nl, vout, cout, &clk);
  }
  // ---- outbox mailboxes + lane results -> records
  if ((r = grow_device(&e->d_oc.p, &e->d_oc.n, (size_t)nl * 4))) return r;
  if ((r = grow_device(&e->d_off.p, &e->d_off.n, (size_t)nl * 4))) return r;
  if ((r = grow_device(&e->d_results.p, &e->d_results.n, (size_t)nl * sizeof(gr_peer_result)))) return r;
  uint32_t* oc = (uint32_t*)e->d_oc.p;
  uint32_t* off = (uint32_t*)e->d_off.p;
  hipLaunchKernelGGL(io::out_counts, dim3(io_grid(nl)), blk, 0, s, vout, nl, S, oc);
  HIPCHK(hipGetLastError());
  if ((r = io_scan(e, oc, off, nl, s))) return r;
  hipLaunchKernelGGL(io::finish_total, dim3(1), dim3(64), 0, s, (const uint32_t*)oc, (const uint32_t*)off, nl,
                     scal + 2);
  hipLaunchKernelGGL(io::pack_results, dim3(io_grid(nl)), blk, 0, s, e->ln, e->st, (const uint32_t*)peer_of_lane,
                     0u, nl, (gr_peer_result*)e->d_results.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_scal + 8, scal + 2, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const uint32_t total = ((uint32_t*)e->h_scal)[2];
  const size_t mbytes = (size_t)total * sizeof(gr_message), rbytes = (size_t)nl * sizeof(gr_peer_result);
  if ((r = grow_device(&e->d_outmsgs.p, &e->d_outmsgs.n, mbytes + 1))) return r;
  if ((r = grow_pinned(&e->h_outmsgs, &e->h_outmsgs_bytes, mbytes + 1))) return r;
  if ((r = grow_pinned(&e->h_results, &e->h_results_bytes, rbytes))) return r;
  if (total) {
    hipLaunchKernelGGL(io::pack_outbox, dim3(io_grid(nl)), blk, 0, s, vout, nl, S, (const uint32_t*)off,
                       (const uint32_t*)peer_of_lane, (gr_message*)e->d_outmsgs.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(e->h_outmsgs, e->d_outmsgs.p, mbytes, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipMemcpyAsync(e->h_results, e->d_results.p, rbytes, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  out->msgs = total ? (gr_message*)e->h_outmsgs : nullptr;
  out->n_msgs = total;
  out->results = (gr_peer_result*)e->h_results;
  out->n_results = nl;
  return GR_OK;
}

int gr_step(gr_engine* e, const gr_inbox* in, gr_outbox* out) {
  if (!e || !in || !out) return GR_EINVAL;
  if ((in->n_msgs && !in->msgs) || (in->n_locals && !in->locals)) return GR_EINVAL;
  if (in->n_msgs + in->n_locals >= 0x80000000ull) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  const uint32_t nm = (uint32_t)in->n_msgs;
  int r;
  if ((r = grow_device(&e->d_msgs.p, &e->d_msgs.n, (size_t)nm * sizeof(gr_message) + 1))) return r;
  if (nm)
    HIPCHK(hipMemcpyAsync(e->d_msgs.p, in->msgs, (size_t)nm * sizeof(gr_message), hipMemcpyHostToDevice, e->stream));
  return step_staged(e, nm, in->locals, (uint32_t)in->n_locals, out);
}

// ---------------------------------------------------------------- wire path
// gr_bind_nodes: the (cluster id, node id) -> engine slot table the wire path
// routes decoded messages with (open addressing, twice the slots, power of two).
int gr_bind_nodes(gr_engine* e, const uint64_t* cluster_ids, const uint64_t* node_ids, uint32_t n) {
  if (!e || (n && (!cluster_ids || !node_ids)) || n > e->cfg.max_peers) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  uint32_t tcap = 64;
  while (tcap < 2 * n) tcap <<= 1;
  std::vector<io::NodeKey> t(tcap);
  for (uint32_t p = 0; p < n; ++p) {
    uint32_t h = io::node_hash(cluster_ids[p], node_ids[p]) & (tcap - 1);
    while (t[h].peer != NOPOS) {
      if (t[h].cluster == cluster_ids[p] && t[h].node == node_ids[p]) return GR_EINVAL;  // listed twice
      h = (h + 1) & (tcap - 1);
    }
    t[h].cluster = cluster_ids[p];
    t[h].node = node_ids[p];
    t[h].peer = p;
  }
  int r;
  if ((r = grow_device(&e->d_nodes.p, &e->d_nodes.n, (size_t)tcap * sizeof(io::NodeKey)))) return r;
  HIPCHK(hipMemcpy(e->d_nodes.p, t.data(), (size_t)tcap * sizeof(io::NodeKey), hipMemcpyHostToDevice));
  e->nodes_cap = tcap;
  return GR_OK;
}

extern "C++" template <int S>
static void launch_route_wire(const grw_message* wm, uint32_t n, const grw_entry* we, uint64_t n_ents,
                              const io::NodeKey* nodes, uint32_t tcap, StateBase st, gr_message* out,
                              uint32_t* flag, uint8_t* why, hipStream_t s) {
  hipLaunchKernelGGL((io::route_wire<S>), dim3(io_grid(n)), dim3(io::kIoBlock), 0, s, wm, n, we, n_ents, nodes, tcap,
                     st, out, flag, why);
}

// The wire path's routing half (gr_step_wire, gr_step_wire_compact): decoded
// records -> routed gr_message records in e->d_msgs (*nm of them), the rest
// listed in *unrouted. Called with e->mu held.
static int wire_route(gr_engine* e, const struct grw_message* d_msgs, size_t n_msgs, const struct grw_entry* d_ents,
                      size_t n_ents, gr_wire_unrouted* unrouted, uint32_t* nm_out) {
  *nm_out = 0;
  unrouted->n = 0;
  unrouted->index = nullptr;
  unrouted->reason = nullptr;
  if (n_msgs && !e->nodes_cap) return GR_ESTATE;  // gr_bind_nodes first
  const uint32_t nw = (uint32_t)n_msgs;
  const hipStream_t s = e->stream;
  const dim3 blk(io::kIoBlock);
  int r;
  if ((r = grow_device(&e->d_msgs.p, &e->d_msgs.n, (size_t)nw * sizeof(gr_message) + 1))) return r;
  uint32_t nm = 0;
  if (nw) {
    // route every decoded message to (slot, sender slot) in a gr_message record,
    // then keep the routed ones in wire order (their arrival order)
    if ((r = grow_device(&e->d_wrec.p, &e->d_wrec.n, (size_t)nw * sizeof(gr_message)))) return r;
    if ((r = grow_device(&e->d_keys.p, &e->d_keys.n, (size_t)nw * 4 + 4))) return r;
    if ((r = grow_device(&e->d_idx.p, &e->d_idx.n, (size_t)nw * 4 + 4))) return r;
    if ((r = grow_device(&e->d_why.p, &e->d_why.n, (size_t)nw + 1))) return r;
    if ((r = grow_device(&e->d_unr.p, &e->d_unr.n, (size_t)nw * 4 + 4))) return r;
    if ((r = grow_device(&e->d_scal.p, &e->d_scal.n, 16))) return r;
    if ((r = grow_pinned(&e->h_scal, &e->h_scal_bytes, 16))) return r;
    uint32_t* flag = (uint32_t*)e->d_keys.p;
    uint32_t* pos = (uint32_t*)e->d_idx.p;
    uint32_t* scal = (uint32_t*)e->d_scal.p;
    switch (e->S) {
      case 1: launch_route_wire<1>(d_msgs, nw, d_ents, n_ents, (const io::NodeKey*)e->d_nodes.p, e->nodes_cap, e->st,
                                   (gr_message*)e->d_wrec.p, flag, (uint8_t*)e->d_why.p, s); break;
      case 3: launch_route_wire<3>(d_msgs, nw, d_ents, n_ents, (const io::NodeKey*)e->d_nodes.p, e->nodes_cap, e->st,
                                   (gr_message*)e->d_wrec.p, flag, (uint8_t*)e->d_why.p, s); break;
      case 5: launch_route_wire<5>(d_msgs, nw, d_ents, n_ents, (const io::NodeKey*)e->d_nodes.p, e->nodes_cap, e->st,
                                   (gr_message*)e->d_wrec.p, flag, (uint8_t*)e->d_why.p, s); break;
      default: launch_route_wire<GR_SMAX>(d_msgs, nw, d_ents, n_ents, (const io::NodeKey*)e->d_nodes.p,
                                          e->nodes_cap, e->st, (gr_message*)e->d_wrec.p, flag,
                                          (uint8_t*)e->d_why.p, s); break;
    }
    HIPCHK(hipGetLastError());
    if ((r = io_scan(e, flag, pos, nw, s))) return r;
    hipLaunchKernelGGL(io::keep_routed, dim3(io_grid(nw)), blk, 0, s, (const gr_message*)e->d_wrec.p,
                       (const uint32_t*)flag, (const uint32_t*)pos, nw, (gr_message*)e->d_msgs.p,
                       (uint32_t*)e->d_unr.p, scal);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(e->h_scal, scal, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    nm = ((uint32_t*)e->h_scal)[0];
    const uint32_t nu = nw - nm;
    if (nu) {  // the messages the host steps with the Go code, in wire order, and why
      if ((r = grow_pinned(&e->h_unr, &e->h_unr_bytes, (size_t)nu * 5))) return r;
      uint32_t* hidx = (uint32_t*)e->h_unr;
      uint8_t* hwhy = e->h_unr + (size_t)nu * 4;
      HIPCHK(hipMemcpyAsync(hidx, e->d_unr.p, (size_t)nu * 4, hipMemcpyDeviceToHost, s));
      std::vector<uint8_t> allwhy(nw);
      HIPCHK(hipMemcpyAsync(allwhy.data(), e->d_why.p, nw, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      for (uint32_t k = 0; k < nu; ++k) hwhy[k] = allwhy[hidx[k]];
      unrouted->n = nu;
      unrouted->index = hidx;
      unrouted->reason = hwhy;
    }
  }
  *nm_out = nm;
  return GR_OK;
}

int gr_step_wire(gr_engine* e, const struct grw_message* d_msgs, size_t n_msgs, const struct grw_entry* d_ents,
                 size_t n_ents, const gr_local_input* locals, size_t n_locals, gr_outbox* out,
                 gr_wire_unrouted* unrouted) {
  if (!e || !out || !unrouted || (n_msgs && !d_msgs) || (n_locals && !locals)) return GR_EINVAL;
  if (n_msgs + n_locals >= 0x80000000ull) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  uint32_t nm;
  int r;
  if ((r = wire_route(e, d_msgs, n_msgs, d_ents, n_ents, unrouted, &nm))) return r;
  return step_staged(e, nm, locals, (uint32_t)n_locals, out);
}

int gr_step_wire_compact(gr_engine* e, const struct grw_message* d_msgs, size_t n_msgs,
                         const struct grw_entry* d_ents, size_t n_ents, const gr_local_input* locals,
                         size_t n_locals, gr_coutbox* out, gr_wire_unrouted* unrouted) {
  if (!e || !out || !unrouted || (n_msgs && !d_msgs) || (n_locals && !locals)) return GR_EINVAL;
  if (n_msgs + n_locals >= 0x80000000ull) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  uint32_t nm;
  int r;
  if ((r = wire_route(e, d_msgs, n_msgs, d_ents, n_ents, unrouted, &nm))) return r;
  return step_staged(e, nm, locals, (uint32_t)n_locals, nullptr, out);
}

// The outbox mailboxes and lane results of the pass just launched, as compact
// records (+ ext records where they do not fit), downloaded into engine-owned
// pinned memory: gr_step_compact_end and gr_step_wire_compact.
static int pack_out_compact(gr_engine* e, uint32_t nl, const SpaceView& vout, gr_coutbox* out, PhaseClock* cl) {
  PhaseClock& clk = *cl;
  const uint32_t S = e->S;
  const hipStream_t s = e->stream;
  const dim3 blk(io::kIoBlock);
  int r;
  uint32_t* scal = (uint32_t*)e->d_scal.p;
  uint32_t* peer_of_lane = e->ln.u32(LR_LANE_PEER);
  // ---- outbox mailboxes + lane results -> compact records (+ ext)
  if ((r = grow_device(&e->d_oc64.p, &e->d_oc64.n, (size_t)nl * 8))) return r;
  if ((r = grow_device(&e->d_off64.p, &e->d_off64.n, (size_t)nl * 8))) return r;
  if ((r = grow_device(&e->d_rx.p, &e->d_rx.n, (size_t)nl * 4))) return r;
  if ((r = grow_device(&e->d_roff.p, &e->d_roff.n, (size_t)nl * 4))) return r;
  if ((r = grow_device(&e->d_results.p, &e->d_results.n, (size_t)nl * sizeof(gr_cresult)))) return r;
  uint64_t* oc = (uint64_t*)e->d_oc64.p;
  uint64_t* off = (uint64_t*)e->d_off64.p;
  uint32_t* rx = (uint32_t*)e->d_rx.p;
  uint32_t* roff = (uint32_t*)e->d_roff.p;
  hipLaunchKernelGGL(io::out_counts_c, dim3(io_grid(nl)), blk, 0, s, vout, e->ln, e->st, nl, S, oc, rx);
  HIPCHK(hipGetLastError());
  if ((r = io_scan64(e, oc, off, nl, s))) return r;
  if ((r = io_scan(e, rx, roff, nl, s))) return r;
  hipLaunchKernelGGL(io::finish_total_c, dim3(1), dim3(64), 0, s, (const uint64_t*)oc, (const uint64_t*)off,
                     (const uint32_t*)rx, (const uint32_t*)roff, nl, scal + 1);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_scal + 4, scal + 1, 12, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  clk.mark("mailboxes+pass+counts");
  const uint32_t total = ((uint32_t*)e->h_scal)[1], text = ((uint32_t*)e->h_scal)[2], rext = ((uint32_t*)e->h_scal)[3];
  const size_t mbytes = (size_t)total * sizeof(gr_cmsg), xbytes = (size_t)text * sizeof(gr_message);
  const size_t rbytes = (size_t)nl * sizeof(gr_cresult), rxbytes = (size_t)rext * sizeof(gr_peer_result);
  if ((r = grow_device(&e->d_outmsgs.p, &e->d_outmsgs.n, mbytes + 1))) return r;
  if ((r = grow_device(&e->d_outext.p, &e->d_outext.n, xbytes + 1))) return r;
  if ((r = grow_device(&e->d_resext.p, &e->d_resext.n, rxbytes + 1))) return r;
  if ((r = grow_pinned(&e->h_outmsgs, &e->h_outmsgs_bytes, mbytes + 1))) return r;
  if ((r = grow_pinned(&e->h_outext, &e->h_outext_bytes, xbytes + 1))) return r;
  if ((r = grow_pinned(&e->h_results, &e->h_results_bytes, rbytes))) return r;
  if ((r = grow_pinned(&e->h_resext, &e->h_resext_bytes, rxbytes + 1))) return r;
  hipLaunchKernelGGL(io::pack_results_c, dim3(io_grid(nl)), blk, 0, s, e->ln, e->st, (const uint32_t*)peer_of_lane,
                     nl, (const uint32_t*)roff, (gr_cresult*)e->d_results.p, (gr_peer_result*)e->d_resext.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_results, e->d_results.p, rbytes, hipMemcpyDeviceToHost, s));
  if (rext) HIPCHK(hipMemcpyAsync(e->h_resext, e->d_resext.p, rxbytes, hipMemcpyDeviceToHost, s));
  if (total) {
    hipLaunchKernelGGL(io::pack_outbox_c, dim3(io_grid(nl)), blk, 0, s, vout, nl, S, (const uint64_t*)off,
                       (const uint32_t*)peer_of_lane, (gr_cmsg*)e->d_outmsgs.p, (gr_message*)e->d_outext.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(e->h_outmsgs, e->d_outmsgs.p, mbytes, hipMemcpyDeviceToHost, s));
    if (text) HIPCHK(hipMemcpyAsync(e->h_outext, e->d_outext.p, xbytes, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  clk.mark("pack+download");
  clk.report();
  out->msgs = total ? (gr_cmsg*)e->h_outmsgs : nullptr;
  out->n_msgs = total;
  out->ext_msgs = text ? (gr_message*)e->h_outext : nullptr;
  out->n_ext_msgs = text;
  out->results = (gr_cresult*)e->h_results;
  out->n_results = nl;
  out->ext_results = rext ? (gr_peer_result*)e->h_resext : nullptr;
  out->n_ext_results = rext;
  return GR_OK;
}

// gr_step with compact records (gpuraft.h gr_cmsg / gr_clocal / gr_cresult):
// the same device passes; records expand in registers on the way in and are
// packed (with ext records for what does not fit) on the way out.
int gr_step_compact_begin(gr_engine* e, const gr_cinbox* in) {
  if (!e || !in) return GR_EINVAL;
  if ((in->n_msgs && !in->msgs) || (in->n_locals && !in->locals) || (in->n_ext_msgs && !in->ext_msgs) ||
      (in->n_ext_locals && !in->ext_locals))
    return GR_EINVAL;
  if (in->n_msgs + in->n_locals >= 0x80000000ull || in->n_ext_msgs >= 0x80000000ull ||
      in->n_ext_locals >= 0x80000000ull)
    return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  if (e->cpend.on) return GR_EINVAL;  // the previous begin was not ended
  GR_REFUSE_PENDING(e);
  PhaseClock clk;  // GR_PHASES=1: per-phase host times on stderr
  const uint32_t S = e->S, cap = e->cfg.max_peers;
  const uint32_t nm = (uint32_t)in->n_msgs, nlc = (uint32_t)in->n_locals;
  const uint32_t nx = (uint32_t)in->n_ext_msgs, nlx = (uint32_t)in->n_ext_locals;
  e->cpend = gr_engine::CPending{};
  if (nm + nlc == 0) {
    e->cpend.on = true;  // an empty pass: _end returns an empty outbox
    e->pending.store(true, std::memory_order_release);
    return GR_OK;
  }
  const hipStream_t s = e->stream;
  const dim3 blk(io::kIoBlock);
  int r;
  // ---- inbox records -> lanes
  if ((r = grow_device(&e->d_msgs.p, &e->d_msgs.n, (size_t)nm * sizeof(gr_cmsg) + 1))) return r;
  if ((r = grow_device(&e->d_locals.p, &e->d_locals.n, (size_t)nlc * sizeof(gr_clocal) + 1))) return r;
  if ((r = grow_device(&e->d_ext.p, &e->d_ext.n, (size_t)nx * sizeof(gr_message) + 1))) return r;
  if ((r = grow_device(&e->d_lext.p, &e->d_lext.n, (size_t)nlx * sizeof(gr_local_input) + 1))) return r;
  if ((r = grow_device(&e->d_mark.p, &e->d_mark.n, (size_t)cap * 4))) return r;
  if ((r = grow_device(&e->d_lop.p, &e->d_lop.n, (size_t)cap * 4))) return r;
  if ((r = grow_device(&e->d_scal.p, &e->d_scal.n, 16))) return r;
  if ((r = grow_pinned(&e->h_scal, &e->h_scal_bytes, 16))) return r;
  uint32_t* mark = (uint32_t*)e->d_mark.p;
  uint32_t* lop = (uint32_t*)e->d_lop.p;
  uint32_t* scal = (uint32_t*)e->d_scal.p;
  io::CInbox ci;
  ci.msgs = (const gr_cmsg*)e->d_msgs.p;
  ci.ext = (const gr_message*)e->d_ext.p;
  ci.loc = (const gr_clocal*)e->d_locals.p;
  ci.lext = (const gr_local_input*)e->d_lext.p;
  ci.n_msgs = nm;
  ci.n_ext = nx;
  ci.n_loc = nlc;
  ci.n_lext = nlx;
  if (nm) HIPCHK(hipMemcpyAsync(e->d_msgs.p, in->msgs, (size_t)nm * sizeof(gr_cmsg), hipMemcpyHostToDevice, s));
  if (nlc) HIPCHK(hipMemcpyAsync(e->d_locals.p, in->locals, (size_t)nlc * sizeof(gr_clocal), hipMemcpyHostToDevice, s));
  if (nx) HIPCHK(hipMemcpyAsync(e->d_ext.p, in->ext_msgs, (size_t)nx * sizeof(gr_message), hipMemcpyHostToDevice, s));
  if (nlx)
    HIPCHK(hipMemcpyAsync(e->d_lext.p, in->ext_locals, (size_t)nlx * sizeof(gr_local_input), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(mark, 0, (size_t)cap * 4, s));
  HIPCHK(hipMemsetAsync(scal, 0, 16, s));
  hipLaunchKernelGGL(io::mark_inputs_c, dim3(io_grid(nm + nlc)), blk, 0, s, ci, S, cap, mark, scal + 1);
  HIPCHK(hipGetLastError());
  if ((r = io_scan(e, mark, lop, cap, s))) return r;
  hipLaunchKernelGGL(io::finish_lanes, dim3(1), dim3(64), 0, s, (const uint32_t*)mark, (const uint32_t*)lop, cap,
                     (const uint32_t*)(scal + 1), scal);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_scal, scal, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  clk.mark("upload+lanes");
  const uint32_t nl = ((uint32_t*)e->h_scal)[0];
  if (((uint32_t*)e->h_scal)[1]) return GR_EINVAL;  // nothing of the pass ran
  e->cpend.on = true;
  e->pending.store(true, std::memory_order_release);
  e->cpend.nm = nm;
  e->cpend.nlc = nlc;
  e->cpend.nx = nx;
  e->cpend.nlx = nlx;
  e->cpend.nl = nl;
  return GR_OK;
}

int gr_step_compact_end(gr_engine* e, gr_coutbox* out) {
  if (!e || !out) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  if (!e->cpend.on) return GR_EINVAL;  // no pass was begun
  const gr_engine::CPending pend = e->cpend;
  e->cpend.on = false;
  // `pending` stays set until this call returns (every path): the pass below
  // still uses the lane rows, bail lists and scratch the flag protects
  struct ClearPending {
    std::atomic<bool>& f;
    ~ClearPending() { f.store(false, std::memory_order_release); }
  } clear_pending{e->pending};
  memset(out, 0, sizeof(*out));
  PhaseClock clk;
  const uint32_t S = e->S, cap = e->cfg.max_peers;
  const uint32_t nm = pend.nm, nlc = pend.nlc, nx = pend.nx, nlx = pend.nlx, nl = pend.nl;
  if (nl == 0) return GR_OK;
  const hipStream_t s = e->stream;
  const dim3 blk(io::kIoBlock);
  int r;
  uint32_t* mark = (uint32_t*)e->d_mark.p;
  uint32_t* lop = (uint32_t*)e->d_lop.p;
  uint32_t* scal = (uint32_t*)e->d_scal.p;
  io::CInbox ci;
  ci.msgs = (const gr_cmsg*)e->d_msgs.p;
  ci.ext = (const gr_message*)e->d_ext.p;
  ci.loc = (const gr_clocal*)e->d_locals.p;
  ci.lext = (const gr_local_input*)e->d_lext.p;
  ci.n_msgs = nm;
  ci.n_ext = nx;
  ci.n_loc = nlc;
  ci.n_lext = nlx;
  (void)nlx;
  uint32_t* peer_of_lane = e->ln.u32(LR_LANE_PEER);
  hipLaunchKernelGGL(io::lane_peers, dim3(io_grid(cap)), blk, 0, s, (const uint32_t*)mark, (const uint32_t*)lop, cap,
                     peer_of_lane);
  HIPCHK(hipGetLastError());
  // ---- mailboxes
  const uint32_t positions = nl * S;
  const size_t space = gr_space_bytes(1, positions, GR_C);
  if ((r = grow_device(&e->d_in.p, &e->d_in.n, space))) return r;
  if ((r = grow_device(&e->d_out.p, &e->d_out.n, space))) return r;
  const SpaceView vin = make_view(e->d_in.p, 1, positions), vout = make_view(e->d_out.p, 1, positions);
  hipLaunchKernelGGL(io::clear_counts, dim3(io_grid(vin.pc)), blk, 0, s, vin, vin.pc);  // the count bytes
  HIPCHK(hipGetLastError());
  if (nm) {
    for (gr_engine::Buf* b : {&e->d_keys, &e->d_idx, &e->d_skeys, &e->d_sidx})
      if ((r = grow_device(&b->p, &b->n, (size_t)nm * 4))) return r;
    hipLaunchKernelGGL(io::msg_keys_c, dim3(io_grid(nm)), blk, 0, s, ci.msgs, nm, (const uint32_t*)lop, nl,
                       (uint32_t*)e->d_keys.p, (uint32_t*)e->d_idx.p);
    HIPCHK(hipGetLastError());
    if ((r = sort_keys(e, nm, positions, s))) return r;
    hipLaunchKernelGGL(io::encode_sorted_c, dim3(io_grid(nm)), blk, 0, s, ci, (const uint32_t*)e->d_skeys.p,
                       (const uint32_t*)e->d_sidx.p, vin);
    HIPCHK(hipGetLastError());
  }
  // ---- locals -> lane rows
  if ((r = grow_device(&e->d_win.p, &e->d_win.n, (size_t)nl * 4))) return r;
  HIPCHK(hipMemsetAsync(e->d_win.p, 0, (size_t)nl * 4, s));
  if (nlc) {
    hipLaunchKernelGGL(io::local_winner_c, dim3(io_grid(nlc)), blk, 0, s, ci.loc, nlc, (const uint32_t*)lop,
                       (uint32_t*)e->d_win.p);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(io::fill_locals_c, dim3(io_grid(nl)), blk, 0, s, ci, (const uint32_t*)e->d_win.p, nl, e->ln);
  HIPCHK(hipGetLastError());
  // ---- the pass
  StepParams kp = base_params(e);
  kp.has_locals = 1;
  kp.has_lane_peer = 1;
  kp.route_mode = RT_IDENTITY;
  kp.in = vin;
  kp.out = vout;
  kp.n_lanes = nl;
  HIPCHK(launch_slots(S, kp, e->bail, e->counters, e->cap, (uint32_t)e->launches++, s, next_timing(e)));
  e->passes++;
  e->locals_set = false;
  e->routes_bound = false;
  if ((r = pack_out_compact(e, nl, vout, out, &clk))) return r;
  return GR_OK;
}

int gr_step_compact(gr_engine* e, const gr_cinbox* in, gr_coutbox* out) {
  if (!e || !in || !out) return GR_EINVAL;
  memset(out, 0, sizeof(*out));
  const int r = gr_step_compact_begin(e, in);
  return r ? r : gr_step_compact_end(e, out);
}

int gr_cinbox_reserve(gr_engine* e, size_t n_msgs, size_t n_ext_msgs, size_t n_locals, size_t n_ext_locals,
                      gr_cinbox* in) {
  if (!e || !in || n_msgs + n_locals >= 0x80000000ull || n_ext_msgs >= 0x80000000ull ||
      n_ext_locals >= 0x80000000ull)
    return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  int r;
  if ((r = grow_pinned(&e->h_inmsgs, &e->h_inmsgs_bytes, n_msgs * sizeof(gr_cmsg) + 1, kInboxPinned))) return r;
  if ((r = grow_pinned(&e->h_inlocals, &e->h_inlocals_bytes, n_locals * sizeof(gr_clocal) + 1, kInboxPinned))) return r;
  if ((r = grow_pinned(&e->h_inext, &e->h_inext_bytes, n_ext_msgs * sizeof(gr_message) + 1, kInboxPinned))) return r;
  if ((r = grow_pinned(&e->h_inlext, &e->h_inlext_bytes, n_ext_locals * sizeof(gr_local_input) + 1, kInboxPinned))) return r;
  in->msgs = (const gr_cmsg*)e->h_inmsgs;
  in->n_msgs = n_msgs;
  in->ext_msgs = (const gr_message*)e->h_inext;
  in->n_ext_msgs = n_ext_msgs;
  in->locals = (const gr_clocal*)e->h_inlocals;
  in->n_locals = n_locals;
  in->ext_locals = (const gr_local_input*)e->h_inlext;
  in->n_ext_locals = n_ext_locals;
  return GR_OK;
}

int gr_release_coutbox(gr_engine* e, gr_coutbox* out) {
  if (!e || !out) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);  // the pinned buffers stay for the next pass
  memset(out, 0, sizeof(*out));
  return GR_OK;
}

int gr_pack_messages(const gr_message* in, size_t n, gr_cmsg* out, gr_message* ext, size_t* n_ext) {
  if ((n && (!in || !out || !ext)) || !n_ext) return GR_EINVAL;
  size_t x = 0;
  for (size_t k = 0; k < n; ++k) {
    if (!host::cmsg_of(in[k], &out[k])) {
      out[k].flags = GR_CM_EXT;
      out[k].aux = (uint32_t)x;
      ext[x++] = in[k];
    }
  }
  *n_ext = x;
  return GR_OK;
}

int gr_unpack_messages(const gr_cmsg* in, size_t n, const gr_message* ext, size_t n_ext, gr_message* out) {
  if (n && (!in || !out)) return GR_EINVAL;
  size_t o = 0;
  for (size_t k = 0; k < n; ++k) {
    if ((in[k].flags & GR_CM_EXT) && (!ext || in[k].aux >= n_ext)) return GR_EINVAL;
    for (uint32_t q = 0; q < host::cmsg_n(in[k]); ++q) out[o++] = host::expand_cmsg(in[k], ext, q);
  }
  return GR_OK;
}

size_t gr_cmsg_count(const gr_cmsg* in, size_t n) {
  size_t t = 0;
  for (size_t k = 0; in && k < n; ++k) t += host::cmsg_n(in[k]);
  return t;
}

int gr_pair_messages(gr_cmsg* c, size_t n, size_t* n_out) {
  if ((n && !c) || !n_out) return GR_EINVAL;
  size_t o = 0;
  for (size_t k = 0; k < n;) {
    gr_cmsg pr;
    if (k + 1 < n && host::pair_of(c[k], c[k + 1], &pr)) {
      c[o++] = pr;
      k += 2;
    } else {
      c[o++] = c[k++];
    }
  }
  *n_out = o;
  return GR_OK;
}

int gr_pack_locals(const gr_local_input* in, size_t n, gr_clocal* out, gr_local_input* ext, size_t* n_ext) {
  if ((n && (!in || !out || !ext)) || !n_ext) return GR_EINVAL;
  size_t x = 0;
  for (size_t k = 0; k < n; ++k) {
    if (!host::clocal_of(in[k], &out[k])) {
      out[k].flags = GR_CL_EXT;
      out[k].ext = (uint32_t)x;
      ext[x++] = in[k];
    }
  }
  *n_ext = x;
  return GR_OK;
}

int gr_inbox_reserve(gr_engine* e, size_t n_msgs, size_t n_locals, gr_inbox* in) {
  if (!e || !in || n_msgs + n_locals >= 0x80000000ull) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  int r;
  if ((r = grow_pinned(&e->h_inmsgs, &e->h_inmsgs_bytes, n_msgs * sizeof(gr_message) + 1, kInboxPinned))) return r;
  if ((r = grow_pinned(&e->h_inlocals, &e->h_inlocals_bytes, n_locals * sizeof(gr_local_input) + 1, kInboxPinned))) return r;
  in->msgs = (const gr_message*)e->h_inmsgs;
  in->n_msgs = n_msgs;
  in->locals = (const gr_local_input*)e->h_inlocals;
  in->n_locals = n_locals;
  return GR_OK;
}

int gr_release_outbox(gr_engine* e, gr_outbox* out) {
  if (!e || !out) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);  // the pinned outbox buffers stay for the next pass
  out->msgs = nullptr;
  out->n_msgs = 0;
  out->results = nullptr;
  out->n_results = 0;
  return GR_OK;
}

static int stat_total(gr_engine* e, uint32_t field, uint64_t* out) {
  std::vector<uint64_t> rows((size_t)e->stats_rows * NSTAT);
  HIPCHK(hipMemcpy(rows.data(), e->stats, rows.size() * 8, hipMemcpyDeviceToHost));
  uint64_t v = 0;
  for (uint32_t b = 0; b < e->stats_rows; ++b) v += rows[(size_t)b * NSTAT + field];
  *out = v;
  return GR_OK;
}

int gr_stats_get(gr_engine* e, gr_stats* out) {
  if (!e || !out) return GR_EINVAL;
  HIPCHK(hipDeviceSynchronize());
  std::vector<uint64_t> rows((size_t)e->stats_rows * NSTAT);
  HIPCHK(hipMemcpy(rows.data(), e->stats, rows.size() * 8, hipMemcpyDeviceToHost));
  memset(out, 0, sizeof(*out));
  out->passes = e->passes;
  for (uint32_t b = 0; b < e->stats_rows; ++b) {
    const uint64_t* row = rows.data() + (size_t)b * NSTAT;
    out->leader_commits += row[ST_LEADER_COMMITS];
    out->follower_commits += row[ST_FOLLOWER_COMMITS];
    out->escalations += row[ST_ESCALATIONS];
    out->msgs_in += row[ST_MSGS_IN];
    out->msgs_out += row[ST_MSGS_OUT];
    out->leader_msgs_in += row[ST_LEADER_MSGS_IN];
    out->leader_msgs_out += row[ST_LEADER_MSGS_OUT];
    out->replicate_entries += row[ST_REPLICATE_ENTRIES];
  }
  return GR_OK;
}

int gr_timing_begin(gr_engine* e) {
  if (!e) return GR_EINVAL;
  HIPCHK(hipDeviceSynchronize());
  free_timings(e);
  e->timings.reserve(1 << 16);  // records are referenced by pointer until the pass is enqueued
  int r = stat_total(e, ST_BAILED, &e->timing_bailed0);
  if (r) return r;
  e->timing = true;
  return GR_OK;
}

int gr_timing_end(gr_engine* e, gr_timing* out) {
  if (!e || !out) return GR_EINVAL;
  HIPCHK(hipDeviceSynchronize());
  memset(out, 0, sizeof(*out));
  for (auto& t : e->timings) {
    float a = 0, b = 0;
    HIPCHK(hipEventElapsedTime(&a, t.ev[0], t.ev[1]));
    HIPCHK(hipEventElapsedTime(&b, t.ev[1], t.ev[2]));
    out->fast_ms += a;
    out->general_ms += b;
    out->passes++;
  }
  uint64_t bailed = 0;
  const int r = stat_total(e, ST_BAILED, &bailed);
  if (r) return r;
  out->bailed_lanes = bailed - e->timing_bailed0;  // lanes that left the lean kernels while timing
  free_timings(e);
  e->timing = false;
  return GR_OK;
}

int gr_stats_reset(gr_engine* e) {
  if (!e) return GR_EINVAL;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemset(e->stats, 0, (size_t)e->stats_rows * NSTAT * 8));
  e->passes = 0;
  return GR_OK;
}

int gr_bind_routes(gr_engine* e, const uint32_t* in_pos, const uint32_t* out_pos, uint32_t n_peers) {
  if (!e || !in_pos || !out_pos || n_peers > e->cfg.max_peers) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);  // against a concurrent compact _begin/_end
  GR_REFUSE_PENDING(e);
  HIPCHK(hipDeviceSynchronize());
  std::vector<uint32_t> base(2 * GR_SMAX * GR_SMAX, NOPOS);
  uint32_t g = 0, rr = 0;
  if (detect_affine_routes(in_pos, out_pos, n_peers, e->S, base.data(), &g, &rr)) {
    HIPCHK(hipMemcpy(e->route_base, base.data(), base.size() * 4, hipMemcpyHostToDevice));
    e->route_mode = is_loopback(base.data(), g, rr, e->S) ? RT_LOOPBACK : RT_AFFINE;
    e->route_g = g;
    e->route_r = rr;
  } else {
    e->route_mode = RT_TABLE;
    e->route_g = 0;
  }
  for (uint32_t j = 0; j < e->S; ++j) {
    HIPCHK(hipMemcpy(e->ln.in_pos() + (size_t)j * e->cap, in_pos + (size_t)j * n_peers, (size_t)n_peers * 4,
                     hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->ln.out_pos() + (size_t)j * e->cap, out_pos + (size_t)j * n_peers,
                     (size_t)n_peers * 4, hipMemcpyHostToDevice));
  }
  e->routes_bound = true;
  return GR_OK;
}

int gr_set_locals(gr_engine* e, const gr_local_input* locals, size_t n) {
  if (!e || (n && !locals) || n >= 0x80000000ull) return GR_EINVAL;
  const uint32_t cap = e->cfg.max_peers;
  for (size_t k = 0; k < n; ++k)
    if (locals[k].peer >= cap) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  HIPCHK(hipDeviceSynchronize());  // a pass in flight on another stream may read the rows
  const hipStream_t s = e->stream;
  int r;
  if ((r = grow_device(&e->d_locals.p, &e->d_locals.n, n * sizeof(gr_local_input) + 1))) return r;
  if ((r = grow_device(&e->d_win.p, &e->d_win.n, (size_t)cap * 4))) return r;
  if (n) HIPCHK(hipMemcpyAsync(e->d_locals.p, locals, n * sizeof(gr_local_input), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(e->d_win.p, 0, (size_t)cap * 4, s));
  const gr_local_input* dloc = (const gr_local_input*)e->d_locals.p;
  if (n) {
    hipLaunchKernelGGL(io::local_winner, dim3(io_grid(n)), dim3(io::kIoBlock), 0, s, dloc, (uint32_t)n,
                       (const uint32_t*)nullptr, (uint32_t*)e->d_win.p);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(io::fill_locals, dim3(io_grid(cap)), dim3(io::kIoBlock), 0, s, dloc,
                     (const uint32_t*)e->d_win.p, cap, e->ln);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  e->locals_set = n > 0;
  bool other = false;
  for (size_t k = 0; k < n && !other; ++k) {
    const gr_local_input& x = locals[k];
    other = local_word(x.ticks, x.quiesced_ticks, x.propose_entries,
                       (x.read_index ? LF_READ_INDEX : 0) | (x.propose_has_config_change ? LF_PROPOSE_CC : 0)) &
            LW_OTHER;
  }
  e->locals_other = other;
  return GR_OK;
}

// One device-resident pass, enqueued on `stream` (e->mu held by the caller).
static int step_device_locked(gr_engine* e, const void* in_space, void* out_space, uint32_t in_chunks,
                              uint32_t in_positions, uint32_t out_chunks, uint32_t out_positions, uint32_t depth,
                              uint32_t n_peers, void* stream) {
  StepParams kp = base_params(e);
  kp.has_locals = e->locals_set ? 1 : 0;
  kp.has_lane_peer = 0;
  kp.route_mode = e->routes_bound ? e->route_mode : RT_IDENTITY;
  kp.route_g = e->route_g;
  kp.route_r = e->route_r;
  kp.route_base = e->route_base;
  kp.route_wu = (kp.route_mode == RT_LOOPBACK || kp.route_mode == RT_AFFINE) && e->route_g % 64 == 0 ? 1 : 0;
  kp.in = make_view(in_space, in_chunks, in_positions, depth);
  kp.out = make_view(out_space, out_chunks, out_positions, depth);
  kp.n_lanes = n_peers;
  // lane = peer here, so a wave's hint carries over between passes
  const size_t hs = hint_stride(e->cap), hf = e->hint_flip++ & 1;
  kp.hints = e->hints + hf * hs;
  kp.hints_out = e->hints + (1 - hf) * hs;
  // the follower instance of its own pays off only when the pass is large (a
  // 10k x 3 pass is launch-bound: one instance there, 24 vs 41 us per pass)
  kp.split = n_peers >= e->split_min ? 1 : 0;
  HIPCHK(launch_slots(e->S, kp, e->bail, e->counters, e->cap, (uint32_t)e->launches++, (hipStream_t)stream,
                      next_timing(e), kp.has_locals && e->locals_other));
  e->passes++;
  return GR_OK;
}

int gr_step_device(gr_engine* e, const void* in_space, void* out_space, uint32_t in_chunks,
                   uint32_t in_positions, uint32_t out_chunks, uint32_t out_positions, uint32_t depth,
                   uint32_t n_peers, void* stream) {
  if (!e || !in_space || !out_space || n_peers > e->cfg.max_peers || depth == 0 || depth > GR_C)
    return GR_EINVAL;
  // the mutex orders this pass after a compact _begin/_end on another thread
  // (uncontended: one lock per pass)
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);  // the pending compact pass owns the lane rows and bail lists
  return step_device_locked(e, in_space, out_space, in_chunks, in_positions, out_chunks, out_positions, depth,
                            n_peers, stream);
}

// A captured sequence of device-resident passes (gpuraft.h gr_graph_*).
struct gr_graph {
  gr_engine* e = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  uint32_t n_passes = 0;
  // the engine's counter-set and hint-set parities the captured pass 0 assumes
  // (launches & 1, hint_flip & 1): a replay at any other parity would read a
  // counter set nobody zeroed and the wrong hint set, so it is refused
  uint32_t launch_par = 0, hint_par = 0;
};

int gr_graph_capture(gr_engine* e, void* space_a, void* space_b, uint32_t n_chunks, uint32_t positions,
                     uint32_t depth, uint32_t n_peers, uint32_t n_passes, gr_graph** out) {
  if (!e || !space_a || !space_b || !out || n_peers > e->cfg.max_peers || depth == 0 || depth > GR_C ||
      n_passes == 0 || (n_passes & 1))
    return GR_EINVAL;
  *out = nullptr;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  if (e->timing) return GR_ESTATE;  // per-pass timing events are not captured
  HIPCHK(hipDeviceSynchronize());   // nothing of the engine in flight while the parities are read
  hipStream_t cs = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  gr_graph* g = new gr_graph();
  g->e = e;
  g->n_passes = n_passes;
  g->launch_par = (uint32_t)(e->launches & 1);
  g->hint_par = (uint32_t)(e->hint_flip & 1);
  // recording runs no pass: the engine's counters are restored afterwards on
  // every path (a failed capture must not leave the parities advanced)
  const uint64_t saved_launches = e->launches, saved_flip = e->hint_flip, saved_passes = e->passes;
  int r = GR_OK;
  if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess) r = GR_EDEVICE;
  // pass k reads space k % 2 and writes the other; the launch and hint parities
  // advance by n_passes (even), so every replay starts where the capture did
  for (uint32_t k = 0; k < n_passes && r == GR_OK; ++k)
    r = step_device_locked(e, (k & 1) ? space_b : space_a, (k & 1) ? space_a : space_b, n_chunks, positions,
                           n_chunks, positions, depth, n_peers, cs);
  hipGraph_t graph = nullptr;
  const hipError_t ce = hipStreamEndCapture(cs, &graph);  // ends the capture on every path
  if (r == GR_OK && (ce != hipSuccess || !graph)) r = GR_EDEVICE;
  if (r == GR_OK && hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0) != hipSuccess) r = GR_EDEVICE;
  g->graph = graph;
  (void)hipStreamDestroy(cs);
  e->launches = saved_launches;
  e->hint_flip = saved_flip;
  e->passes = saved_passes;
  if (r != GR_OK) {
    gr_graph_destroy(g);
    return r;
  }
  *out = g;
  return GR_OK;
}

int gr_graph_replay(gr_graph* g, void* stream) {
  if (!g || !g->exec) return GR_EINVAL;
  std::lock_guard<std::mutex> guard(g->e->mu);
  GR_REFUSE_PENDING(g->e);
  gr_engine* e = g->e;
  // passes run between replays must come in even numbers (gpuraft.h)
  if ((uint32_t)(e->launches & 1) != g->launch_par || (uint32_t)(e->hint_flip & 1) != g->hint_par)
    return GR_ESTATE;
  HIPCHK(hipGraphLaunch(g->exec, (hipStream_t)stream));
  e->launches += g->n_passes;
  e->hint_flip += g->n_passes;
  e->passes += g->n_passes;
  return GR_OK;
}

void gr_graph_destroy(gr_graph* g) {
  if (!g) return;
  if (g->exec) (void)hipGraphExecDestroy(g->exec);
  if (g->graph) (void)hipGraphDestroy(g->graph);
  delete g;
}

int gr_collect_results(gr_engine* e, uint32_t first, gr_peer_result* out, size_t n) {
  if (!e || (n && !out) || (uint64_t)first + n > e->cfg.max_peers) return GR_EINVAL;
  if (n == 0) return GR_OK;
  std::lock_guard<std::mutex> guard(e->mu);
  GR_REFUSE_PENDING(e);
  HIPCHK(hipDeviceSynchronize());
  const size_t bytes = n * sizeof(gr_peer_result);
  int r;
  if ((r = grow_device(&e->d_results.p, &e->d_results.n, bytes))) return r;
  hipLaunchKernelGGL(io::pack_results, dim3(io_grid(n)), dim3(io::kIoBlock), 0, e->stream, e->ln, e->st,
                     (const uint32_t*)nullptr, first, (uint32_t)n, (gr_peer_result*)e->d_results.p);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, e->d_results.p, bytes, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return GR_OK;
}

#ifdef GR_COVERAGE
// Coverage build only (libgpuraft_cover.so): per-branch hit counts (gr_cover.h).
int gr_coverage_read(uint64_t* out, uint32_t n) {
  if (!out || n < CV_N) return GR_EINVAL;
  HIPCHK(hipDeviceSynchronize());
  for (uint32_t k = 0; k < CV_N; ++k) out[k] = 0;
  HIPCHK(cover_read<1>(out));  // every kernel translation unit keeps its own counters
  HIPCHK(cover_read<3>(out));
  HIPCHK(cover_read<5>(out));
  HIPCHK(cover_read<8>(out));
  return (int)CV_N;
}
const char* gr_coverage_names() {
#define GR_COVER_NAME(x) #x ","
  return GR_COVER_IDS(GR_COVER_NAME);
#undef GR_COVER_NAME
}
#endif

}  // extern "C"

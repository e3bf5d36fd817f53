// SPDX-License-Identifier: Apache-2.0
//
// C-ABI implementation (include/dpgpu.h): contexts, table publication and
// burst submission on HIP streams.
//
// Table publication mirrors the reference's lock-free reader handles
// (left-right for FIB / NAT, ArcSwap Slot for flow-filter / ACL,
// SURVEY.md §1): dp_tables_publish compiles and uploads a new image, then
// swaps one per-device shared pointer under a mutex.  Every burst keeps a
// reference to the image it launched with until a completion event of that
// burst has fired (polled without blocking at the context's next burst), so
// an old image is released only after the last burst reading it has ended.
// A released image's memory goes to a per-device graveyard and is freed by
// the publishing (mgmt) thread -- hipFree synchronises the device, so it never
// runs on a worker's burst path.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dpgpu.h"
#include "dp_flows_rt.h"
#include "dp_tables.h"

extern "C" int dpk_launch_pipeline(const uint8_t *img_base, const void *image_dev, uint8_t *buf,
                                   uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                                   dp_pkt_meta_t *meta, uint32_t n, uint64_t *stats, uint64_t *stats_part,
                                   int v6w, int ctx, hipStream_t stream);
extern "C" int dpk_acl_classify(const uint8_t *img_base, const void *image_dev, const dp_acl_key_t *keys,
                                dp_acl_result_t *out, uint32_t n, hipStream_t stream);
extern "C" int dpk_ff_classify(const uint8_t *img_base, const void *image_dev, const dp_ff_input_t *in,
                               dp_ff_result_t *out, uint32_t n, int stage, hipStream_t stream);
extern "C" int dpk_mark_failed(const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n,
                               hipStream_t stream);
extern "C" int dpk_stage_expand(const uint8_t *cin, const uint32_t *pos, const dp_pkt_in_t *in, uint8_t *buf,
                                uint32_t n, hipStream_t stream);
extern "C" int dpk_stage_collect(const uint8_t *buf, const uint32_t *pos, const dp_pkt_in_t *in, uint8_t *cout,
                                 uint32_t grow, uint32_t n, hipStream_t stream);
extern "C" int dpk_launch_pipeline_flows(const uint8_t *img_base, const void *image_dev, uint8_t *buf,
                                         uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                                         dp_pkt_meta_t *meta, uint32_t n, uint64_t *stats, uint64_t *stats_part,
                                         const void *fc_host, hipStream_t stream, hipStream_t side,
                                         hipEvent_t fork, hipEvent_t fork2, hipEvent_t join, int fork_at);

namespace {

thread_local std::string g_err;

int fail(int rc, const char *what, hipError_t e = hipSuccess) {
  g_err = what;
  if (e != hipSuccess) {
    g_err += ": ";
    g_err += hipGetErrorString(e);
  }
  return rc;
}

// How many distinct HIP runtimes (libamdhip64 files) the process maps.  Two
// appear when another library brings its own copy after this one loaded
// (PyTorch bundles one and asks for it by the unversioned name, which this
// library's libamdhip64.so.7 does not answer): two HIP and two HSA runtimes
// then each manage the process's one KFD state, and host-memory copies of
// one went unwritten.  1 when /proc is unreadable.
int hip_runtimes_mapped() {
  FILE *f = std::fopen("/proc/self/maps", "r");
  if (!f) return 1;
  std::vector<std::string> seen;
  char line[4096];
  while (std::fgets(line, sizeof line, f)) {
    const char *p = std::strchr(line, '/');
    if (!p) continue;
    std::string path(p);
    while (!path.empty() && (path.back() == '\n' || path.back() == ' ')) path.pop_back();
    const size_t b = path.rfind('/');
    if (path.compare(b + 1, 14, "libamdhip64.so") != 0) continue;
    if (std::find(seen.begin(), seen.end(), path) == seen.end()) seen.push_back(path);
  }
  std::fclose(f);
  return seen.empty() ? 1 : (int)seen.size();
}

}  // namespace

int dpr_fail(int rc, const char *what, hipError_t e) { return fail(rc, what, e); }

namespace {

struct DeviceTables;
DeviceTables &dev_tables(int device);

// Device memory of retired images, freed by the publishing thread.
struct Graveyard {
  std::mutex mu;
  std::vector<uint8_t *> dead;
};
std::mutex g_grave_mu;
std::map<int, std::unique_ptr<Graveyard>> g_grave;

Graveyard &graveyard(int device) {
  std::lock_guard<std::mutex> lk(g_grave_mu);
  auto &p = g_grave[device];
  if (!p) p.reset(new Graveyard());
  return *p;
}

void bury(int device, uint8_t *p) {
  Graveyard &gy = graveyard(device);
  std::lock_guard<std::mutex> lk(gy.mu);
  gy.dead.push_back(p);
}

// hipFree the retired images of `device` (publish / destroy only).
void drain_graveyard(int device) {
  std::vector<uint8_t *> dead;
  {
    Graveyard &gy = graveyard(device);
    std::lock_guard<std::mutex> lk(gy.mu);
    dead.swap(gy.dead);
  }
  if (dead.empty()) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  for (uint8_t *p : dead) (void)hipFree(p);
  (void)hipSetDevice(prev);
}

struct DevImage {
  int device = 0;
  uint8_t *dev = nullptr;
  dpd::Image im{};
  uint64_t im_off = 0;  // the Image descriptor, uploaded after the table bytes
  // the masquerade config the flow tables build their allocators from, and
  // this build's serial (a table syncs once per build)
  std::shared_ptr<const dpd::MasqConfig> masq;
  uint64_t serial = 0;
  ~DevImage() {
    if (dev) bury(device, dev);  // freed later, off the burst path
  }
};

struct DeviceTables {
  std::mutex mu;
  // publishes of one device, one at a time: each builds on the lineage (the
  // port-forwarding entry ids) the previous one stored
  std::mutex pub_mu;
  std::shared_ptr<DevImage> cur;
  dpd::PfLineage pf;  // the port-forwarding entries of `cur` (PortFwTable::update lineage)
  // the flow tables attached to contexts of this device (attach count each):
  // a publish syncs their masquerade allocators (update_nat_allocator runs
  // when the config is applied).  Order: pub_mu, then reg_mu, then a table's mu.
  std::mutex reg_mu;
  std::map<dp_flow_table *, int> fts;
};
std::atomic<uint64_t> g_serial{1};
std::atomic<uint32_t> g_nat_seq{0};  // dpf_debug_nat_sequential
std::atomic<uint32_t> g_flows_full{0};  // dpf_debug_flows_full
std::atomic<uint32_t> g_last_lean{0};   // dpf_debug_last_lean
std::atomic<uint32_t> g_no_ctx{0};      // dpf_debug_no_ctx
// where the NAT pass forks the replay of the records off the allocating lane
// to the side stream: 0 never (one replay after the lane), 1 after the
// resolve, 2 after the lane's plan, 3 the steady refreshes after dp_nat_prep
// and the rest after the lane's plan (dpf_debug_replay_fork; DPGPU_REPLAY_FORK)
std::atomic<int> g_replay_fork{-1};
int replay_fork() {
  int v = g_replay_fork.load(std::memory_order_relaxed);
  if (v < 0) {
    const char *e = getenv("DPGPU_REPLAY_FORK");
    v = e && *e >= '0' && *e <= '3' && !e[1] ? *e - '0' : 2;
    g_replay_fork.store(v, std::memory_order_relaxed);
  }
  return v;
}

std::mutex g_dev_mu;
std::map<int, std::unique_ptr<DeviceTables>> g_dev;

DeviceTables &dev_tables(int device) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto &p = g_dev[device];
  if (!p) p.reset(new DeviceTables());
  return *p;
}

// One launched burst: the image it reads and its completion event.
struct InFlight {
  std::shared_ptr<DevImage> img;
  hipEvent_t done = nullptr;
};

// DoneReason partial histograms: a small ring of buffers, one per launch.
// A slot is reused only after the launch that used it (kernel + reduce) has
// completed: the new launch's stream waits on the slot's event, so bursts on
// different streams never share partial counters.
constexpr int kPartSlots = 4;

// Host-origin bursts are moved in chunks of at least kHostChunk packets on
// kHostStreams streams, so one chunk's device-to-host copy, the next one's
// kernel and the one after's host-to-device copy overlap (PCIe is full
// duplex).
constexpr uint32_t kHostChunk = 65536;
constexpr int kHostStreams = 3;
class HostPool;
struct PartSlot {
  uint64_t *part = nullptr;
  hipEvent_t used = nullptr;
  bool armed = false;
};

}  // namespace

struct dp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::deque<InFlight> inflight;     // bursts not yet known complete
  std::vector<hipEvent_t> spare;     // recycled completion events
  PartSlot parts[kPartSlots];
  int next_part = 0;
  // host-path staging
  uint8_t *d_buf = nullptr;
  uint64_t d_buf_cap = 0;
  dp_pkt_in_t *d_in = nullptr;
  dp_pkt_out_t *d_out = nullptr;
  dp_pkt_meta_t *d_meta = nullptr;
  uint64_t *d_stats = nullptr;
  // the classifiers alone on host memory (dp_acl_classify, dp_ff_classify):
  // device inputs and results, and their pinned host staging (grown as needed)
  void *cls_dev = nullptr;
  void *cls_host = nullptr;
  size_t cls_cap = 0;
  uint32_t cap_n = 0;
  uint32_t *d_pos = nullptr;           // staged copies: span positions (16-byte units)
  // staged copies: pinned host side (records, positions, packed spans in and
  // out) and the packed spans on the device
  dp_pkt_in_t *h_in = nullptr;
  dp_pkt_out_t *h_out = nullptr;
  dp_pkt_meta_t *h_meta = nullptr;
  uint32_t *h_pos = nullptr;
  uint8_t *h_cin = nullptr, *h_cout = nullptr, *d_cin = nullptr, *d_cout = nullptr;
  uint64_t cin_cap = 0, cout_cap = 0;
  std::vector<hipEvent_t> chunk_ev;    // per chunk: its D2H has landed
  hipStream_t hs[kHostStreams] = {};   // host-path copy/compute streams
  hipEvent_t hev[kHostStreams + 1] = {};
  bool host_streams = false;
  int host_path = DP_HOST_AUTO;        // dp_ctx_set_option(DP_OPT_HOST_PATH)
  // flow table (dp_ctx_attach_flow_table) and the per-launch flow scratch:
  // invalidation events and flow-dependent ACL verdicts; a launch waits for
  // the previous flows launch before reusing it
  dp_flow_table *ft = nullptr;
  // dp_process_mbufs: pinned, device-mapped burst records
  dp_pkt_in_t *mb_in = nullptr;
  dp_pkt_out_t *mb_out = nullptr;
  dp_pkt_meta_t *mb_meta = nullptr;
  uint32_t mb_cap = 0;
  FlowScratch fl_ev, fl_sens;
  // port forwarding scratch (dpf::FlowCtx pf*): records, counters, packet ->
  // record, bitmaps (kept zero between bursts), order, replaced fills
  FlowScratch pf_req, pf_cnt, pf_of, pf_bits, pf_order, pf_repl, mq_rel, lane_order, lane_plan, lane_res, lane_key, steady, adm, adm_blk;
  // the NAT pass's connection tables and the keyed index of replaced fills:
  // entries carry the burst's tag, so they are zeroed only when allocated
  FlowScratch grp_tab, grp_head, grp_next, grp_list, repl, dup_tab;
  uint32_t burst_tag = 0;
  uint64_t pf_bits_n = 0;
  hipEvent_t fl_used = nullptr;
  bool fl_armed = false;
  // the NAT pass's side stream (lowest priority): the replay of the records
  // off the allocating lane runs on it beside the lane (fork / join events)
  hipStream_t side = nullptr;
  hipEvent_t side_fork = nullptr, side_fork2 = nullptr, side_join = nullptr;
  bool side_tried = false;
  uint64_t clock = 0;                  // dp_ctx_set_option(DP_OPT_CLOCK)
  // host threads of the staged-copy path, the context's own: a staged burst
  // waits for its own chunks only, never for another worker's
  std::unique_ptr<HostPool> pool;
};

namespace {

// Drop the image references of bursts that have completed (non-blocking).
void reap(dp_ctx *c) {
  while (!c->inflight.empty()) {
    InFlight &f = c->inflight.front();
    if (f.done && hipEventQuery(f.done) == hipErrorNotReady) break;
    if (f.done) c->spare.push_back(f.done);
    c->inflight.pop_front();
  }
}

hipEvent_t take_event(dp_ctx *c) {
  if (!c->spare.empty()) {
    hipEvent_t e = c->spare.back();
    c->spare.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

// Phase timing of the staged-copy path, printed when DPGPU_HOST_TRACE is set
// (diagnostics for the host-inclusive rate).
struct HostTrace {
  const bool on = getenv("DPGPU_HOST_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::string s;
  void mark(const char *what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    s += std::string(what) + " " + std::to_string(std::chrono::duration<double, std::micro>(now - t).count()) + " us; ";
    t = now;
  }
  void done(uint32_t n, uint32_t threads, uint32_t chunks) {
    if (on) fprintf(stderr, "[dpgpu host] n=%u threads=%u chunks=%u: %s\n", n, threads, chunks, s.c_str());
  }
};

// The staged path's byte moves.  A span goes into pinned staging that only
// the DMA engine reads: streaming stores (no read for ownership of the
// staging lines, no cache pollution), fenced before the copies are enqueued.
// A frame comes back from staging the DMA engine wrote: 16-byte moves.
void put_span(uint8_t *dst, const uint8_t *src, uint64_t units) {  // dst 16-byte aligned
  for (uint64_t k = 0; k < units; k++)
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 16 * k),
                     _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 16 * k)));
}
void put_frame(uint8_t *dst, const uint8_t *src, uint32_t len) {
  uint32_t k = 0;
  for (; k + 16 <= len; k += 16)
    _mm_storeu_si128(reinterpret_cast<__m128i *>(dst + k), _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + k)));
  if (k < len) memcpy(dst + k, src + k, len - k);
}

// Host threads for a burst's gather / write-back: one per 32K packets, at
// most the machine's threads (capped at 16).
uint32_t host_threads(uint32_t n) {
  const uint32_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  return std::max(1u, std::min(hw, n / 32768));
}
// A pool of host threads for the staged-copy path's gather and write-back,
// one per context, created on its first staged burst and kept until the
// context is destroyed (thread creation per burst cost more than the gather
// itself).  run(parts, f) calls f(t) for every t in
// [0, parts) -- the caller takes part of the work -- and returns when all
// are done; concurrent callers take turns.
class HostPool {
 public:
  void run(uint32_t parts, const std::function<void(uint32_t)> &f) {
    if (parts <= 1) {
      f(0u);
      return;
    }
    std::lock_guard<std::mutex> turn(run_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      while (th_.size() + 1 < parts) th_.emplace_back([this] { work(); });
      job_ = &f;
      parts_ = parts;
      next_ = 0;
      pending_ = parts;
      gen_++;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }

 private:
  void drain() {  // take parts until none is left
    for (;;) {
      uint32_t t;
      const std::function<void(uint32_t)> *f;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!job_ || next_ >= parts_) return;
        t = next_++;
        f = job_;
      }
      (*f)(t);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_all();
    }
  }
  void work() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      drain();
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(uint32_t)> *job_ = nullptr;
  uint32_t parts_ = 0, next_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

template <class F>
void par_for(dp_ctx *c, uint32_t parts, F &&f) {
  if (!c->pool) c->pool.reset(new HostPool());
  c->pool->run(parts, std::function<void(uint32_t)>(std::forward<F>(f)));
}

// Every per-packet array of the host paths (the device records and span
// positions, their pinned host sides), grown together to at least n packets:
// the staged and the sharded paths share them, so one capacity covers all.
hipError_t ensure_records(dp_ctx *c, uint32_t n) {
  if (n <= c->cap_n) return hipSuccess;
  (void)hipStreamSynchronize(c->stream);
  for (void *p : {(void *)c->d_in, (void *)c->d_out, (void *)c->d_meta, (void *)c->d_pos}) if (p) (void)hipFree(p);
  for (void *p : {(void *)c->h_in, (void *)c->h_out, (void *)c->h_meta, (void *)c->h_pos}) if (p) (void)hipHostFree(p);
  c->d_in = nullptr; c->d_out = nullptr; c->d_meta = nullptr; c->d_pos = nullptr;
  c->h_in = nullptr; c->h_out = nullptr; c->h_meta = nullptr; c->h_pos = nullptr;
  c->cap_n = 0;
  hipError_t e;
  if ((e = hipMalloc(&c->d_in, sizeof(dp_pkt_in_t) * n)) != hipSuccess ||
      (e = hipMalloc(&c->d_out, sizeof(dp_pkt_out_t) * n)) != hipSuccess ||
      (e = hipMalloc(&c->d_meta, sizeof(dp_pkt_meta_t) * n)) != hipSuccess ||
      (e = hipMalloc(&c->d_pos, sizeof(uint32_t) * n)) != hipSuccess ||
      (e = hipHostMalloc(&c->h_in, sizeof(dp_pkt_in_t) * n)) != hipSuccess ||
      (e = hipHostMalloc(&c->h_out, sizeof(dp_pkt_out_t) * n)) != hipSuccess ||
      (e = hipHostMalloc(&c->h_meta, sizeof(dp_pkt_meta_t) * n)) != hipSuccess ||
      (e = hipHostMalloc(&c->h_pos, sizeof(uint32_t) * n)) != hipSuccess)
    return e;
  c->cap_n = n;
  return hipSuccess;
}

// Every packet of a failed burst is InternalFailure (dpgpu.h conventions,
// SURVEY.md §5 failure detection); host arrays.
void mark_failed_host(const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    if (out) {
      dp_pkt_out_t o{};
      o.off = in ? in[i].off : 0;
      o.len = in ? in[i].len : 0;
      o.done = DP_DONE_INTERNAL_FAILURE;
      out[i] = o;
    }
    if (meta) {
      dp_pkt_meta_t m{};
      m.fib_entry = m.acl_rule = 0xffffffffu;
      m.flow_ref = DP_FLOW_NONE;
      meta[i] = m;
    }
  }
}

}  // namespace

extern "C" {

uint32_t dp_abi_version(void) { return DPGPU_ABI_VERSION; }

// Test hook (not part of dpgpu.h): the classifiers' host-memory copies -- 0
// pinned staging, stream-ordered on the context's stream (the default); 1 the
// round-5 path, hipMemcpyAsync between pageable memory and stream-ordered
// allocations (scripts/dev/hip_runtimes_diag.py reproduces its anomaly).
// Test hook (not part of dpgpu.h): the HIP runtimes this process maps
// (dp_ctx_create refuses more than one)
int dpd_debug_hip_runtimes(void) { return hip_runtimes_mapped(); }

static std::atomic<int> g_cls_copies{0};
void dpd_debug_classify_copies(int mode) { g_cls_copies.store(mode == 1 ? 1 : 0, std::memory_order_relaxed); }

const char *dp_last_error(void) { return g_err.c_str(); }

int dp_ctx_create(int device_ordinal, dp_ctx_t **out) {
  if (!out) return fail(DP_EINVAL, "null out");
  if (hip_runtimes_mapped() > 1 && !std::getenv("DPGPU_ALLOW_TWO_HIP_RUNTIMES"))
    return fail(DP_ENOTSUP, "two HIP runtimes mapped in this process (load the one PyTorch bundles before "
                            "libdpgpu.so, or none: DESIGN.md §5)");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(DP_ENODEV, "no HIP device", e);
  if (device_ordinal < 0 || device_ordinal >= ndev) return fail(DP_ENODEV, "bad device ordinal");
  std::unique_ptr<dp_ctx> c(new dp_ctx());
  c->device = device_ordinal;
  if ((e = hipSetDevice(device_ordinal)) != hipSuccess) return fail(DP_EIO, "hipSetDevice", e);
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(DP_EIO, "hipStreamCreate", e);
  if ((e = hipMalloc(&c->d_stats, sizeof(uint64_t) * DP_DONE_COUNT)) != hipSuccess)
    return fail(DP_ENOMEM, "hipMalloc stats", e);
  const size_t part_bytes = sizeof(uint64_t) * DP_DONE_COUNT * DPD_STAT_SLOTS;
  for (auto &ps : c->parts) {
    if ((e = hipMalloc(&ps.part, part_bytes)) != hipSuccess) return fail(DP_ENOMEM, "hipMalloc stats partials", e);
    if ((e = hipMemset(ps.part, 0, part_bytes)) != hipSuccess) return fail(DP_EIO, "clear stats partials", e);
    if ((e = hipEventCreateWithFlags(&ps.used, hipEventDisableTiming)) != hipSuccess)
      return fail(DP_EIO, "hipEventCreate", e);
  }
  *out = c.release();
  return 0;
}

int dp_ctx_destroy(dp_ctx_t *c) {
  if (!c) return DP_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto &f : c->inflight) {
    if (f.done) {
      (void)hipEventSynchronize(f.done);
      (void)hipEventDestroy(f.done);
    }
  }
  c->inflight.clear();
  for (hipEvent_t e : c->spare) (void)hipEventDestroy(e);
  for (auto &ps : c->parts) {
    if (ps.used) { (void)hipEventSynchronize(ps.used); (void)hipEventDestroy(ps.used); }
    if (ps.part) (void)hipFree(ps.part);
  }
  if (c->d_buf) (void)hipFree(c->d_buf);
  if (c->d_in) (void)hipFree(c->d_in);
  if (c->d_out) (void)hipFree(c->d_out);
  if (c->d_meta) (void)hipFree(c->d_meta);
  for (void *p : {(void *)c->d_pos, (void *)c->d_cin, (void *)c->d_cout}) if (p) (void)hipFree(p);
  for (void *p : {(void *)c->h_in, (void *)c->h_out, (void *)c->h_meta, (void *)c->h_pos, (void *)c->h_cin, (void *)c->h_cout})
    if (p) (void)hipHostFree(p);
  for (hipEvent_t e : c->chunk_ev) (void)hipEventDestroy(e);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->cls_dev) (void)hipFree(c->cls_dev);
  if (c->cls_host) (void)hipHostFree(c->cls_host);
  c->fl_ev.release();
  c->fl_sens.release();
  for (FlowScratch *x : {&c->pf_req, &c->pf_cnt, &c->pf_of, &c->pf_bits, &c->pf_order, &c->pf_repl, &c->mq_rel,
                         &c->lane_order, &c->lane_plan, &c->lane_res, &c->lane_key, &c->steady, &c->adm, &c->adm_blk, &c->dup_tab,
                         &c->grp_tab, &c->grp_head, &c->grp_next, &c->grp_list, &c->repl})
    x->release();
  if (c->ft) {
    DeviceTables &dt = dev_tables(c->device);
    std::lock_guard<std::mutex> lk(dt.reg_mu);
    auto it = dt.fts.find(c->ft);
    if (it != dt.fts.end() && --it->second <= 0) dt.fts.erase(it);
  }
  if (c->mb_in) (void)hipHostFree(c->mb_in);
  if (c->mb_out) (void)hipHostFree(c->mb_out);
  if (c->mb_meta) (void)hipHostFree(c->mb_meta);
  if (c->fl_used) (void)hipEventDestroy(c->fl_used);
  if (c->side) { (void)hipStreamSynchronize(c->side); (void)hipStreamDestroy(c->side); }
  if (c->side_fork) (void)hipEventDestroy(c->side_fork);
  if (c->side_fork2) (void)hipEventDestroy(c->side_fork2);
  if (c->side_join) (void)hipEventDestroy(c->side_join);
  for (auto &h : c->hs) if (h) { (void)hipStreamSynchronize(h); (void)hipStreamDestroy(h); }
  for (auto &e : c->hev) if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  const int dev = c->device;
  delete c;
  drain_graveyard(dev);
  return 0;
}

int dp_tables_publish(dp_ctx_t *c, const dp_tables_desc_t *tables) {
  if (!c || !tables) return fail(DP_EINVAL, "null argument");
  dpd::BuiltImage bi;
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> publishing(dt.pub_mu);
  dpd::PfLineage pf;
  {
    std::lock_guard<std::mutex> lk(dt.mu);
    pf = dt.pf;
  }
  int rc = dpd::build_image(tables, bi, &pf);
  if (rc) return fail(rc, "table compile rejected the descriptors");
  (void)hipSetDevice(c->device);
  drain_graveyard(c->device);  // images no burst reads any more
  auto img = std::make_shared<DevImage>();
  img->device = c->device;
  // the kernel reads the Image descriptor from HBM (scalar loads where used)
  // instead of taking it by value: 100+ kernel-argument SGPRs would spill
  img->im_off = (bi.bytes.size() + 63) & ~(uint64_t)63;
  bi.bytes.resize(img->im_off + sizeof(dpd::Image));
  memcpy(bi.bytes.data() + img->im_off, &bi.im, sizeof(dpd::Image));
  hipError_t e = hipMalloc(&img->dev, bi.bytes.size());
  if (e != hipSuccess) return fail(DP_ENOMEM, "hipMalloc table image", e);
  if ((e = hipMemcpy(img->dev, bi.bytes.data(), bi.bytes.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(DP_EIO, "upload table image", e);
  img->im = bi.im;
  img->masq = bi.masq;
  img->serial = g_serial++;
  std::shared_ptr<DevImage> old;
  {
    std::lock_guard<std::mutex> lk(dt.mu);
    old = dt.cur;
    dt.cur = img;
    dt.pf = std::move(pf);
  }
  // the attached flow tables' allocators follow the new config now (a table
  // attached later syncs at its first burst).  Every table is tried; the first
  // failure is returned, with the new image already published: a table that
  // failed keeps its old allocator and tries again at its next burst (which
  // fails the burst, whole, while the sync does)
  {
    std::lock_guard<std::mutex> reg(dt.reg_mu);
    int first = 0;
    for (auto &kv : dt.fts) {
      std::lock_guard<std::mutex> lk(kv.first->mu);
      const int r = dpf_masq_sync(kv.first, img->masq, img->im.genid, img->serial);
      if (r && !first) first = r;
    }
    if (first) return fail(first, "masquerade allocator update (the new tables are published)");
  }
  // `old` is retired here only if no in-flight burst still references it
  return 0;
}

int64_t dp_tables_genid(const dp_ctx_t *c) {
  if (!c) return -1;
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> lk(dt.mu);
  return dt.cur ? dt.cur->im.genid : -1;
}

uint64_t dp_tables_device_bytes(const dp_ctx_t *c) {
  if (!c) return 0;
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> lk(dt.mu);
  return dt.cur ? dt.cur->im.bytes : 0;
}

static std::shared_ptr<DevImage> current(dp_ctx_t *c) {
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> lk(dt.mu);
  return dt.cur;
}

static int launch_burst(dp_ctx_t *c, uint8_t *dev_buf, uint64_t buf_bytes, const dp_pkt_in_t *dev_in,
                        dp_pkt_out_t *dev_out, dp_pkt_meta_t *dev_meta, uint32_t n, uint64_t *dev_stats,
                        void *stream) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!dev_in || !dev_out) return fail(DP_EINVAL, "null burst descriptors");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  reap(c);
  auto img = current(c);
  if (!dev_buf || ((uintptr_t)dev_buf & 15) || !img) {
    // whole-burst failure: every packet InternalFailure
    (void)dpk_mark_failed(dev_in, dev_out, dev_meta, n, s);
    return !img ? fail(DP_ENOTABLES, "no tables published") : fail(DP_EINVAL, "bad burst buffer");
  }
  uint64_t *part = nullptr;
  PartSlot *ps = nullptr;
  if (dev_stats) {
    ps = &c->parts[c->next_part];
    c->next_part = (c->next_part + 1) % kPartSlots;
    if (ps->armed && hipStreamWaitEvent(s, ps->used, 0) != hipSuccess) return fail(DP_EIO, "stream wait");
    part = ps->part;
  }
  int rc;
  if (c->ft) {
    // the flows variant: FlowLookup on the attached table and the flow-aware
    // stages, with this launch's event / verdict scratch; in the table's one
    // order (dp_flows_rt.h): after every earlier management call and every
    // earlier flows burst of any context attached to the table
    dp_flow_table *ft = c->ft;
    std::lock_guard<std::mutex> lk(ft->mu);
    // the table's allocator follows the image's masquerade config
    if (ft->mq_serial != img->serial) {
      if ((rc = dpf_masq_sync(ft, img->masq, img->im.genid, img->serial))) {
        (void)dpk_mark_failed(dev_in, dev_out, dev_meta, n, s);
        return fail(rc, "masquerade allocator update");
      }
    }
    if (c->fl_armed && hipStreamWaitEvent(s, c->fl_used, 0) != hipSuccess) return fail(DP_EIO, "stream wait");
    if (ft->burst_armed && hipStreamWaitEvent(s, ft->last_burst, 0) != hipSuccess)
      return fail(DP_EIO, "stream wait (flow table)");
    dpf::FlowCtx fc{};
    fc.slots = ft->slots;
    fc.mask = ft->mask;
    fc.max_probe = 0;
    fc.n = n;
    // (slot, state) events: <= 2 per packet in the first pass, <= 6 in the
    // sequential NAT pass (invalidations and their hand-over at refills)
    fc.events = static_cast<uint32_t *>(c->fl_ev.get(sizeof(uint32_t) * (1 + 16 * (uint64_t)n)));
    fc.sens = static_cast<uint32_t *>(c->fl_sens.get(sizeof(uint32_t) * 8 + sizeof(dpf::SensRec) * (uint64_t)n));
    fc.genid = img->im.genid;
    fc.tmeta = ft->d_meta;
    fc.capacity = ft->capacity;
    fc.hard = ft->nslots - ft->nslots / 8;
    fc.now = c->clock;
    // port forwarding: the bitmaps stay zero between bursts (dp_nat_prep
    // clears what it reads); grown bitmaps start zeroed.  dp_nat_prep reads
    // the bitmap a whole 1024-packet region (32 words) at a time, so it spans
    // whole regions; the summary words sit after them
    const uint64_t words = ((uint64_t)n + 1023) / 1024 * 32, sum_words = ((uint64_t)n + 32767) / 32768;
    fc.pf = static_cast<dpf::PfReq *>(c->pf_req.get(sizeof(dpf::PfReq) * (uint64_t)n));
    fc.pf_cnt = static_cast<uint32_t *>(c->pf_cnt.get(sizeof(uint32_t) * DPF_CNT_WORDS));
    fc.pf_of = static_cast<uint32_t *>(c->pf_of.get(sizeof(uint32_t) * (uint64_t)n));
    fc.pf_order = static_cast<uint32_t *>(c->pf_order.get(sizeof(uint32_t) * (uint64_t)n));
    fc.pf_repl = static_cast<uint32_t *>(c->pf_repl.get(sizeof(uint32_t) * 8 * ((uint64_t)n + 1)));
    // masquerade: the allocator, and the allocations of replaced fills (at
    // most two fills per packet) released after the sequential pass
    fc.mq = ft->mq;
    fc.mq_gen = ft->mq_gen;
    fc.mq_rel = static_cast<uint32_t *>(c->mq_rel.get(sizeof(uint32_t) * 4 * ((uint64_t)n + 1)));
    // the NAT pass's connections: a hash table of at least 2n slots, a list
    // link per record, the slots claimed; the replaced fills (<= 2 per
    // record) keyed at load <= 1/2.  Tagged by the burst: zeroed only when
    // (re)allocated, never cleared between bursts
    uint64_t gt = 1024;
    while (gt < 2 * (uint64_t)n) gt <<= 1;
    uint64_t rt = 1024;
    while (rt < 4 * (uint64_t)n + 2) rt <<= 1;
    auto zeroed = [&](FlowScratch &x, size_t bytes) -> void * {
      const bool fresh = bytes > x.cap;
      void *p = x.get(bytes);
      if (p && fresh && hipMemsetAsync(p, 0, x.cap, s) != hipSuccess) return nullptr;
      return p;
    };
    fc.grp_tab = static_cast<unsigned long long *>(zeroed(c->grp_tab, sizeof(uint64_t) * gt));
    fc.grp_head = static_cast<unsigned long long *>(zeroed(c->grp_head, sizeof(uint64_t) * gt));
    fc.dup_tab = static_cast<unsigned long long *>(zeroed(c->dup_tab, sizeof(uint64_t) * gt));
    fc.grp_next = static_cast<unsigned long long *>(c->grp_next.get(sizeof(uint64_t) * ((uint64_t)n + 1)));
    fc.grp_list = static_cast<uint32_t *>(c->grp_list.get(sizeof(uint32_t) * ((uint64_t)n + 1)));
    fc.repl = static_cast<uint4 *>(zeroed(c->repl, sizeof(uint4) * rt));
    // a table grown since the last burst holds the smallest power of two
    // that fits (its mask names that many entries, zeroed)
    fc.grp_mask = (uint32_t)(std::min({c->grp_tab.cap, c->grp_head.cap, c->dup_tab.cap}) / sizeof(uint64_t) - 1);
    fc.rmask = (uint32_t)(c->repl.cap / sizeof(uint4) - 1);
    if (++c->burst_tag == 0) {  // tags wrapped: every entry is zeroed again
      c->burst_tag = 1;
      if (fc.grp_tab) (void)hipMemsetAsync(fc.grp_tab, 0, c->grp_tab.cap, s);
      if (fc.grp_head) (void)hipMemsetAsync(fc.grp_head, 0, c->grp_head.cap, s);
      if (fc.dup_tab) (void)hipMemsetAsync(fc.dup_tab, 0, c->dup_tab.cap, s);
      if (fc.repl) (void)hipMemsetAsync(fc.repl, 0, c->repl.cap, s);
    }
    fc.burst = c->burst_tag;
    fc.force_seq = g_nat_seq.load(std::memory_order_relaxed);
    // the flows variant without stateful NAT: an image without it, on a table
    // no such image's burst ever ran on (only those bursts make NAT state),
    // no v6 windows (the lean units leave those lookups out) and context
    // tables that fit the lean units' LDS copy
    if (img->im.snat) ft->snat_seen = true;
    fc.lean = !ft->snat_seen && !img->im.v6w_c && !img->im.v6w_fib && img->im.ctx_bytes &&
              !g_flows_full.load(std::memory_order_relaxed);
    g_last_lean.store(fc.lean, std::memory_order_relaxed);
    fc.ctx = img->im.ctx_bytes != 0 && !g_no_ctx.load(std::memory_order_relaxed);
    // (two bitmaps: the packets that reached the NAT stages, then the
    // masquerading burst's allocating lane, dp_nat_lane_order)
    if (words + sum_words > c->pf_bits_n) {
      c->pf_bits.release();
      c->pf_bits_n = 0;
      void *b = c->pf_bits.get(2 * sizeof(uint32_t) * (words + sum_words));
      if (b && hipMemsetAsync(b, 0, 2 * sizeof(uint32_t) * (words + sum_words), s) == hipSuccess)
        c->pf_bits_n = words + sum_words;
    }
    fc.pf_bits = static_cast<uint32_t *>(c->pf_bits.p);
    fc.pf_sum = fc.pf_bits ? fc.pf_bits + words : nullptr;
    fc.lane_bits = fc.pf_bits ? fc.pf_bits + words + sum_words : nullptr;
    fc.lane_sum = fc.lane_bits ? fc.lane_bits + words : nullptr;
    fc.lane_order = static_cast<uint32_t *>(c->lane_order.get(sizeof(uint32_t) * ((uint64_t)n + 1)));
    // the masquerade split's lane scratch (208 B a packet) only for an image
    // that configures masquerade; without it a masquerading record (a flow
    // that kept masquerade state from an earlier configuration) sends the
    // burst to the one-lane pass (pfw::nat_mode)
    if (img->im.masq) {
      fc.lane_plan = static_cast<uint4 *>(c->lane_plan.get(128 * ((uint64_t)n + 1)));
      fc.lane_res = static_cast<uint4 *>(c->lane_res.get(32 * ((uint64_t)n + 1)));
      fc.lane_key = static_cast<uint4 *>(c->lane_key.get(48 * ((uint64_t)n + 1)));
    }
    const bool lane_ok = !img->im.masq || (fc.lane_plan && fc.lane_res && fc.lane_key);
    fc.steady = static_cast<unsigned long long *>(c->steady.get(8 * ((uint64_t)n / 64 + 2)));
    fc.adm = static_cast<uint32_t *>(c->adm.get(sizeof(uint32_t) * ((uint64_t)n + 1)));
    fc.adm_blk = static_cast<uint32_t *>(c->adm_blk.get(sizeof(uint32_t) * 1024));
    if (!fc.events || !fc.sens || !fc.pf || !fc.pf_cnt || !fc.pf_of || !fc.pf_order || !fc.pf_repl || !fc.mq_rel ||
        !fc.lane_order || !lane_ok || !fc.steady || !fc.dup_tab || !fc.adm || !fc.adm_blk ||
        !fc.grp_tab || !fc.grp_head || !fc.grp_next || !fc.grp_list || !fc.repl ||
        c->pf_bits_n < words + sum_words) {
      (void)dpk_mark_failed(dev_in, dev_out, dev_meta, n, s);
      return fail(DP_ENOMEM, "flow burst scratch");
    }
    const int fork_at = fc.lean ? 0 : replay_fork();
    if (fork_at && !c->side_tried) {
      // (made once; without it the replay runs after the lane, on `s`)
      c->side_tried = true;
      int lo = 0, hi = 0;
      if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = 0;
      if (hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, lo) != hipSuccess ||
          hipEventCreateWithFlags(&c->side_fork, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&c->side_fork2, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&c->side_join, hipEventDisableTiming) != hipSuccess)
        (void)hipGetLastError();
    }
    rc = dpk_launch_pipeline_flows(img->dev, img->dev + img->im_off, dev_buf, buf_bytes, dev_in, dev_out,
                                   dev_meta, n, dev_stats, part, &fc, s, fork_at ? c->side : nullptr,
                                   c->side_fork, c->side_fork2, c->side_join, fork_at);
    if (!rc) {
      if (!c->fl_used && hipEventCreateWithFlags(&c->fl_used, hipEventDisableTiming) != hipSuccess)
        return fail(DP_EIO, "hipEventCreate");
      (void)hipEventRecord(c->fl_used, s);
      c->fl_armed = true;
      if (hipEventRecord(ft->last_burst, s) == hipSuccess) ft->burst_armed = true;
    }
  } else {
    rc = dpk_launch_pipeline(img->dev, img->dev + img->im_off, dev_buf, buf_bytes, dev_in, dev_out, dev_meta, n,
                             dev_stats, part, img->im.v6w_c || img->im.v6w_fib,
                             img->im.ctx_bytes != 0 && !g_no_ctx.load(std::memory_order_relaxed), s);
  }
  if (rc) {
    hipError_t e = hipGetLastError();
    (void)dpk_mark_failed(dev_in, dev_out, dev_meta, n, s);
    return fail(DP_EIO, "kernel launch failed", e);
  }
  if (ps) {
    (void)hipEventRecord(ps->used, s);
    ps->armed = true;
  }
  InFlight f;
  f.img = img;
  f.done = take_event(c);
  if (f.done) (void)hipEventRecord(f.done, s);
  c->inflight.push_back(std::move(f));
  return 0;
}

int dp_process_burst_device(dp_ctx_t *c, uint8_t *dev_buf, uint64_t buf_bytes,
                            const dp_pkt_in_t *dev_in, dp_pkt_out_t *dev_out, dp_pkt_meta_t *dev_meta,
                            uint32_t n, uint64_t *dev_stats, void *stream) {
  return launch_burst(c, dev_buf, buf_bytes, dev_in, dev_out, dev_meta, n, dev_stats, stream);
}

int dp_acl_classify_device(dp_ctx_t *c, const dp_acl_key_t *dev_keys, dp_acl_result_t *dev_out, uint32_t n,
                           void *stream) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!dev_keys || !dev_out) return fail(DP_EINVAL, "null keys / results");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  reap(c);
  auto img = current(c);
  if (!img) return fail(DP_ENOTABLES, "no tables published");
  if (dpk_acl_classify(img->dev, img->dev + img->im_off, dev_keys, dev_out, n, s))
    return fail(DP_EIO, "ACL classify launch failed", hipGetLastError());
  // the image stays alive until the lookups that read it complete
  InFlight f;
  f.img = img;
  f.done = take_event(c);
  if (f.done) (void)hipEventRecord(f.done, s);
  c->inflight.push_back(std::move(f));
  return 0;
}

// A classifier over keys and results in host memory: the keys staged through
// pinned memory onto the device, the lookups, the results back -- every copy
// ordered on the context's stream, one synchronisation at the end.
// `launch(dev_in, dev_out)` enqueues the lookups on the context's stream.
static int classify_host(dp_ctx_t *c, const void *in, size_t in_bytes, void *out, size_t out_bytes,
                         const std::function<int(const void *, void *)> &launch) {
  (void)hipSetDevice(c->device);
  hipError_t e;
  const size_t in_al = (in_bytes + 255) & ~(size_t)255, need = in_al + out_bytes;
  if (g_cls_copies.load(std::memory_order_relaxed) == 1) {
    // the round-5 path: stream-ordered allocations, asynchronous copies
    // to and from pageable memory
    void *d = nullptr;
    if ((e = hipMallocAsync(&d, need, c->stream)) != hipSuccess) return fail(DP_ENOMEM, "classify buffers", e);
    int rc = 0;
    if ((e = hipMemcpyAsync(d, in, in_bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
      rc = fail(DP_EIO, "classify keys copy", e);
    if (!rc) rc = launch(d, (uint8_t *)d + in_al);
    if (!rc && (e = hipMemcpyAsync(out, (uint8_t *)d + in_al, out_bytes, hipMemcpyDeviceToHost, c->stream)) !=
                   hipSuccess)
      rc = fail(DP_EIO, "classify results copy", e);
    (void)hipFreeAsync(d, c->stream);
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess && !rc) rc = fail(DP_EIO, "classify", e);
    return rc;
  }
  if (need > c->cls_cap) {
    // (the context's stream first: an earlier lookup may still use them)
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return fail(DP_EIO, "classify", e);
    if (c->cls_dev) (void)hipFree(c->cls_dev);
    if (c->cls_host) (void)hipHostFree(c->cls_host);
    c->cls_dev = c->cls_host = nullptr;
    c->cls_cap = 0;
    const size_t cap = std::max(need, (size_t)1 << 20);
    if ((e = hipMalloc(&c->cls_dev, cap)) != hipSuccess || (e = hipHostMalloc(&c->cls_host, cap)) != hipSuccess)
      return fail(DP_ENOMEM, "classify buffers", e);
    c->cls_cap = cap;
  }
  uint8_t *hin = static_cast<uint8_t *>(c->cls_host), *din = static_cast<uint8_t *>(c->cls_dev);
  // (the staging is the context's: nothing of an earlier call is in flight
  // once this call's copies are enqueued behind it on the same stream -- but
  // the host may only overwrite it after that call's results were read,
  // which the synchronisation below guarantees)
  std::memcpy(hin, in, in_bytes);
  if ((e = hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return fail(DP_EIO, "classify keys copy", e);
  int rc = launch(din, din + in_al);
  if (!rc && (e = hipMemcpyAsync(hin + in_al, din + in_al, out_bytes, hipMemcpyDeviceToHost, c->stream)) !=
                 hipSuccess)
    rc = fail(DP_EIO, "classify results copy", e);
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess && !rc) rc = fail(DP_EIO, "classify", e);
  if (!rc) std::memcpy(out, hin + in_al, out_bytes);
  return rc;
}

int dp_acl_classify(dp_ctx_t *c, const dp_acl_key_t *keys, dp_acl_result_t *out, uint32_t n) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!keys || !out) return fail(DP_EINVAL, "null keys / results");
  return classify_host(c, keys, sizeof(dp_acl_key_t) * (size_t)n, out, sizeof(dp_acl_result_t) * (size_t)n,
                       [&](const void *dk, void *dr) {
                         return dp_acl_classify_device(c, static_cast<const dp_acl_key_t *>(dk),
                                                       static_cast<dp_acl_result_t *>(dr), n, c->stream);
                       });
}

int dp_acl_key_from_match(const uint8_t *match, uint32_t key_size, uint32_t stride, uint32_t n,
                          dp_acl_key_t *out) {
  if (key_size != DP_ACL_MATCH_KEY_V4 && key_size != DP_ACL_MATCH_KEY_V6)
    return fail(DP_EINVAL, "ACL match key: 21 (v4) or 45 (v6) bytes");
  if (stride < key_size) return fail(DP_EINVAL, "ACL match key stride shorter than the key");
  if (n && (!match || !out)) return fail(DP_EINVAL, "null keys / output");
  const uint32_t al = key_size == DP_ACL_MATCH_KEY_V4 ? 4 : 16;
  auto be32 = [](const uint8_t *b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; };
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t *b = match + (size_t)i * stride;
    dp_acl_key_t k{};
    k.proto = b[0];
    k.src_vni = be32(b + 1);
    k.dst_vni = be32(b + 5);
    k.family = al == 4 ? 4 : 6;
    std::memcpy(k.src, b + 9, al);
    std::memcpy(k.dst, b + 9 + al, al);
    k.sport = (uint16_t)(b[9 + 2 * al] << 8 | b[10 + 2 * al]);
    k.dport = (uint16_t)(b[11 + 2 * al] << 8 | b[12 + 2 * al]);
    out[i] = k;
  }
  return 0;
}

int dp_acl_classify_match(dp_ctx_t *c, const uint8_t *match, uint32_t key_size, uint32_t stride, uint32_t n,
                          dp_acl_result_t *out) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  std::vector<dp_acl_key_t> keys(n);
  const int rc = dp_acl_key_from_match(match, key_size, stride, n, keys.data());
  if (rc || !n) return rc;
  return dp_acl_classify(c, keys.data(), out, n);
}

namespace {
int ff_classify_device(dp_ctx_t *c, const dp_ff_input_t *dev_in, dp_ff_result_t *dev_out, uint32_t n, int stage,
                       void *stream) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!dev_in || !dev_out) return fail(DP_EINVAL, "null inputs / results");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  reap(c);
  auto img = current(c);
  if (!img) return fail(DP_ENOTABLES, "no tables published");
  if (dpk_ff_classify(img->dev, img->dev + img->im_off, dev_in, dev_out, n, stage, s))
    return fail(DP_EIO, "flow-filter classify launch failed", hipGetLastError());
  InFlight f;
  f.img = img;
  f.done = take_event(c);
  if (f.done) (void)hipEventRecord(f.done, s);
  c->inflight.push_back(std::move(f));
  return 0;
}
int ff_classify_host(dp_ctx_t *c, const dp_ff_input_t *in, dp_ff_result_t *out, uint32_t n, int stage) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!in || !out) return fail(DP_EINVAL, "null inputs / results");
  return classify_host(c, in, sizeof(dp_ff_input_t) * (size_t)n, out, sizeof(dp_ff_result_t) * (size_t)n,
                       [&](const void *di, void *dr) {
                         return ff_classify_device(c, static_cast<const dp_ff_input_t *>(di),
                                                   static_cast<dp_ff_result_t *>(dr), n, stage, c->stream);
                       });
}
}  // namespace

int dp_ff_classify_device(dp_ctx_t *c, const dp_ff_input_t *dev_in, dp_ff_result_t *dev_out, uint32_t n,
                          void *stream) {
  return ff_classify_device(c, dev_in, dev_out, n, 0, stream);
}

int dp_ff_classify(dp_ctx_t *c, const dp_ff_input_t *in, dp_ff_result_t *out, uint32_t n) {
  return ff_classify_host(c, in, out, n, 0);
}

int dp_ff_key_from_match(int table, const uint8_t *match, uint32_t key_size, uint32_t stride, uint32_t n,
                         dp_ff_input_t *out) {
  uint32_t al;
  if (table == DP_FF_REMOTE && (key_size == DP_FF_REMOTE_KEY_V4 || key_size == DP_FF_REMOTE_KEY_V6))
    al = key_size == DP_FF_REMOTE_KEY_V4 ? 4 : 16;
  else if (table == DP_FF_LOCAL && (key_size == DP_FF_LOCAL_KEY_V4 || key_size == DP_FF_LOCAL_KEY_V6))
    al = key_size == DP_FF_LOCAL_KEY_V4 ? 4 : 16;
  else
    return fail(DP_EINVAL, "flow-filter match key: remote 15 / 27, local 16 / 28 bytes");
  if (stride < key_size) return fail(DP_EINVAL, "flow-filter match key stride shorter than the key");
  if (n && (!match || !out)) return fail(DP_EINVAL, "null keys / output");
  auto be32 = [](const uint8_t *b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; };
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t *b = match + (size_t)i * stride;
    dp_ff_input_t k{};
    k.proto = b[0];
    k.src_vni = be32(b + 1);
    k.dst_vni = be32(b + 5);
    k.src_family = k.dst_family = al == 4 ? 4 : 6;
    const uint16_t port = (uint16_t)(b[9 + al] << 8 | b[10 + al]);
    if (table == DP_FF_REMOTE) {  // RemoteKey: proto, src_vni, dst_vni (GateVni), dst_ip, dst_port
      std::memcpy(k.dst, b + 9, al);
      k.dport = port;
    } else {  // LocalKey: proto, src_vni, dst_vni, src_ip, src_port, gate
      std::memcpy(k.src, b + 9, al);
      k.sport = port;
      k.gate = b[11 + al];
    }
    out[i] = k;
  }
  return 0;
}

int dp_ff_classify_match(dp_ctx_t *c, int table, const uint8_t *match, uint32_t key_size, uint32_t stride,
                         uint32_t n, dp_ff_result_t *out) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  std::vector<dp_ff_input_t> in(n);
  const int rc = dp_ff_key_from_match(table, match, key_size, stride, n, in.data());
  if (rc || !n) return rc;
  return ff_classify_host(c, in.data(), out, n, table);
}

int dp_ctx_attach_flow_table(dp_ctx_t *c, dp_flow_table_t *ft) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (ft && ft->device != c->device) return fail(DP_EINVAL, "flow table on another device");
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> reg(dt.reg_mu);
  if (c->ft) {
    auto it = dt.fts.find(c->ft);
    if (it != dt.fts.end() && --it->second <= 0) dt.fts.erase(it);
  }
  if (ft) dt.fts[ft]++;
  c->ft = ft;
  return 0;
}

// Test hook (not part of dpgpu.h): 1 runs every burst's NAT pass on one lane
// in packet order (the parallel pass's reference in the parity tests and A/Bs);
// 2 runs masquerading bursts' split pass with every allocation on the
// allocating lane alone (no wave batches); 3 runs port-forwarding bursts
// without room for every pair on one lane (no admission pass); 4 runs mixed
// bursts on one lane (no mode 5); 5 runs the allocating lane without its bulk
// serve (every allocation in the lane's steps); 6 the bulk serve with every
// block opened by one lane (no wave-wide open).
void dpf_debug_nat_sequential(int on) {
  g_nat_seq.store(on >= 1 && on <= 6 ? (uint32_t)on : 0u, std::memory_order_relaxed);
}
// Test hook (not part of dpgpu.h): the context's last flows burst's NAT-pass
// counters (dp_flow.h FlowCtx::pf_cnt: the mode that ran, the split pass's
// lane records and allocations), up to `n` words.
int dpf_debug_nat_counters(dp_ctx_t *c, uint32_t *out, uint32_t n) {
  if (!c || !out) return DP_EINVAL;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (!c->pf_cnt.p) return DP_EINVAL;
  if (n > DPF_CNT_WORDS) n = DPF_CNT_WORDS;
  return hipMemcpy(out, c->pf_cnt.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost) == hipSuccess ? (int)n : DP_EIO;
}
// Test hook (not part of dpgpu.h): 1 runs every flows burst through the full
// flows variant (stateful NAT compiled in) even where the lean one serves.
void dpf_debug_flows_full(int on) { g_flows_full.store(on ? 1u : 0u, std::memory_order_relaxed); }
// Test hook (not part of dpgpu.h): 1 runs the non-flow pipeline without the
// LDS copy of the context tables even where they fit (A/Bs, parity of both).
void dpf_debug_no_ctx(int on) { g_no_ctx.store(on ? 1u : 0u, std::memory_order_relaxed); }
// Test hook (not part of dpgpu.h): where the NAT pass forks the replay off the
// allocating lane (0 never, 1 after the resolve, 2 after the lane's plan, 3
// the steady refreshes after dp_nat_prep and the rest after the plan;
// -1 back to DPGPU_REPLAY_FORK / the default, 2).
void dpf_debug_replay_fork(int at) { g_replay_fork.store(at >= 0 && at <= 3 ? at : -1, std::memory_order_relaxed); }
// Test hook: 1 if the last flows burst launched ran the lean variant.
int dpf_debug_last_lean() { return (int)g_last_lean.load(std::memory_order_relaxed); }

// Test hook (not part of dpgpu.h): the context's last flows burst's NAT pass
// -- its counters (pf_cnt[0..7]) and up to `max` records (dpf::PfReq).
// With `next` (u64 per record) and `heads` (u64 per connection): the
// records' list links and each connection's list head.
int dpf_debug_nat_records(dp_ctx_t *c, uint32_t *cnt8, void *recs, uint32_t max, uint64_t *next,
                          uint64_t *heads) {
  if (!c || !cnt8) return DP_EINVAL;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (!c->pf_cnt.p) return DP_EINVAL;
  if (hipMemcpy(cnt8, c->pf_cnt.p, sizeof(uint32_t) * 8, hipMemcpyDeviceToHost) != hipSuccess) return DP_EIO;
  const uint32_t k = cnt8[0] < max ? cnt8[0] : max;
  if (k && recs && hipMemcpy(recs, c->pf_req.p, sizeof(dpf::PfReq) * k, hipMemcpyDeviceToHost) != hipSuccess)
    return DP_EIO;
  if (k && next && hipMemcpy(next, c->grp_next.p, sizeof(uint64_t) * k, hipMemcpyDeviceToHost) != hipSuccess)
    return DP_EIO;
  if (heads && cnt8[4] && c->grp_list.p) {
    std::vector<uint32_t> lst(cnt8[4]);
    std::vector<uint64_t> tab(c->grp_head.cap / 8);
    if (hipMemcpy(lst.data(), c->grp_list.p, 4 * lst.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(tab.data(), c->grp_head.p, c->grp_head.cap, hipMemcpyDeviceToHost) != hipSuccess)
      return DP_EIO;
    for (size_t e = 0; e < lst.size(); e++) heads[e] = tab[lst[e]];
  }
  return 0;
}
uint32_t dpf_debug_nat_record_bytes(void) { return sizeof(dpf::PfReq); }

// A flow table being destroyed leaves every device's registry.
void dpr_forget_flow_table(dp_flow_table *ft) {
  DeviceTables &dt = dev_tables(ft->device);
  std::lock_guard<std::mutex> reg(dt.reg_mu);
  dt.fts.erase(ft);
}

// The device-visible address of pinned, device-mapped host memory (the
// caller's hipHostMalloc'd / registered buffers), nullptr for anything else.
static void *mapped_ptr(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  const char *base = static_cast<const char *>(a.hostPointer ? a.hostPointer : p);
  return static_cast<char *>(a.devicePointer) + (static_cast<const char *>(p) - base);
}

int dp_ctx_set_option(dp_ctx_t *c, int option, int64_t value) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (option == DP_OPT_HOST_PATH) {
    if (value < DP_HOST_AUTO || value > DP_HOST_ZERO_COPY) return fail(DP_EINVAL, "bad host path mode");
    c->host_path = (int)value;
    return 0;
  }
  if (option == DP_OPT_CLOCK) {
    if (value < 0) return fail(DP_EINVAL, "negative clock");
    c->clock = (uint64_t)value;
    return 0;
  }
  return fail(DP_EINVAL, "unknown option");
}

int dp_process_burst(dp_ctx_t *c, uint8_t *buf, uint64_t buf_bytes, const dp_pkt_in_t *in,
                     dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n, uint64_t *stats) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!buf || !in || !out) {
    mark_failed_host(in, out, meta, n);
    return fail(DP_EINVAL, "null burst buffers");
  }
  for (uint32_t i = 0; i < n; i++)
    if (in[i].off < DP_HEADROOM || (uint64_t)in[i].off + in[i].len > buf_bytes) {
      mark_failed_host(in, out, meta, n);
      return fail(DP_EINVAL, "frame outside the burst buffer / headroom");
    }
  (void)hipSetDevice(c->device);
  hipError_t e;
  auto bail = [&](int rc, const char *what, hipError_t err) {
    mark_failed_host(in, out, meta, n);
    return fail(rc, what, err);
  };
  // Zero-copy: when the burst buffer and the record arrays are pinned,
  // device-mapped host memory, the kernel reads the frames and records over
  // PCIe and writes the rewritten header spans and records back in place --
  // only the bytes the path touches cross the link (window chunks in, the
  // rewritten span and the 16-byte record out), no staging copies.
  if (c->host_path != DP_HOST_COPY) {
    uint64_t end = 0;
    for (uint32_t i = 0; i < n; i++) end = std::max<uint64_t>(end, ((uint64_t)in[i].off + in[i].len + 15) & ~15ull);
    uint8_t *db = static_cast<uint8_t *>(mapped_ptr(buf));
    const dp_pkt_in_t *din = static_cast<const dp_pkt_in_t *>(mapped_ptr(in));
    dp_pkt_out_t *dout = static_cast<dp_pkt_out_t *>(mapped_ptr(out));
    dp_pkt_meta_t *dmeta = meta ? static_cast<dp_pkt_meta_t *>(mapped_ptr(meta)) : nullptr;
    const bool zc = db && din && dout && (!meta || dmeta) && !((uintptr_t)db & 15) && end <= buf_bytes;
    if (zc) {
      hipStream_t s = c->stream;
      if (stats && (e = hipMemsetAsync(c->d_stats, 0, sizeof(uint64_t) * DP_DONE_COUNT, s)) != hipSuccess)
        return bail(DP_EIO, "memset stats", e);
      int rc = dp_process_burst_device(c, db, buf_bytes, din, dout, dmeta, n, stats ? c->d_stats : nullptr, s);
      uint64_t hstats[DP_DONE_COUNT];
      if (!rc && stats && (e = hipMemcpyAsync(hstats, c->d_stats, sizeof(hstats), hipMemcpyDeviceToHost, s)) != hipSuccess)
        rc = fail(DP_EIO, "D2H stats", e);
      if ((e = hipStreamSynchronize(s)) != hipSuccess && !rc) rc = fail(DP_EIO, "stream sync", e);
      if (rc) { mark_failed_host(in, out, meta, n); return rc; }
      if (stats) for (int k = 0; k < DP_DONE_COUNT; k++) stats[k] += hstats[k];
      return 0;
    }
    if (c->host_path == DP_HOST_ZERO_COPY) return bail(DP_EINVAL, "zero-copy needs pinned, mapped, 16-byte aligned buffers", hipSuccess);
  }
  // Staged copies (memory the device cannot map): only the frames cross the
  // link.  Host threads pack each packet's 16-byte span [off & ~15,
  // (off + len + 15) & ~15) back to back into pinned staging.  Per chunk of
  // >= kHostChunk packets, on kHostStreams streams: the spans, their
  // positions and the records go H2D, dp_stage_expand puts every span at its
  // own offset of a device copy of the burst buffer, the pipeline runs, and
  // dp_stage_collect packs each span -- grown in front by the headroom (DP_HEADROOM) when an
  // output may start before its frame (VXLAN encap) -- for the D2H.  Host
  // threads then write each delivered frame back in place.  PCIe carries the
  // frame spans, 16 B of record each way (+ the meta records) and, with
  // encap, DP_HEADROOM bytes of headroom out (a VXLAN-over-IPv6 outer stack is 70 B).  With a flow table the burst is one launch.
  const uint64_t need = ((buf_bytes + 15) & ~15ull) + 16;
  if (need > c->d_buf_cap) {
    if (c->d_buf) { (void)hipStreamSynchronize(c->stream); (void)hipFree(c->d_buf); }
    c->d_buf = nullptr;
    if ((e = hipMalloc(&c->d_buf, need)) != hipSuccess) { c->d_buf_cap = 0; return bail(DP_ENOMEM, "hipMalloc burst", e); }
    c->d_buf_cap = need;
  }
  if ((e = ensure_records(c, n)) != hipSuccess) return bail(DP_ENOMEM, "burst records (device / pinned)", e);
  dp_pkt_meta_t *dm = meta ? c->d_meta : nullptr;
  hipStream_t s = c->stream;
  const uint32_t grow = [&] {
    auto img = current(c);
    return img && img->im.may_encap ? (uint32_t)DP_HEADROOM : 0u;
  }();
  // spans: per-thread sums, then positions (16-byte units) and the gather
  HostTrace tr;
  const uint32_t T = host_threads(n);
  std::vector<uint64_t> acc(T + 1, 0);
  par_for(c, T, [&](uint32_t t) {
    uint64_t sum = 0;
    for (uint32_t i = (uint32_t)((uint64_t)n * t / T), b = (uint32_t)((uint64_t)n * (t + 1) / T); i < b; i++)
      sum += ((in[i].off + in[i].len + 15u) >> 4) - (in[i].off >> 4);
    acc[t + 1] = sum;
  });
  for (uint32_t t = 0; t < T; t++) acc[t + 1] += acc[t];
  const uint64_t units = acc[T];
  if (units >= (1ull << 32)) return bail(DP_EINVAL, "burst spans beyond 64 GiB", hipSuccess);
  const uint64_t in_bytes = 16 * units, out_bytes = in_bytes + (uint64_t)grow * n;
  if (in_bytes > c->cin_cap || out_bytes > c->cout_cap) {
    (void)hipStreamSynchronize(c->stream);
    for (void *p : {(void *)c->d_cin, (void *)c->d_cout}) if (p) (void)hipFree(p);
    for (void *p : {(void *)c->h_cin, (void *)c->h_cout}) if (p) (void)hipHostFree(p);
    c->d_cin = c->d_cout = c->h_cin = c->h_cout = nullptr;
    c->cin_cap = c->cout_cap = 0;
    const uint64_t ci = std::max<uint64_t>(in_bytes, 1 << 20), co = std::max<uint64_t>(out_bytes, 1 << 20);
    if ((e = hipMalloc(&c->d_cin, ci)) != hipSuccess || (e = hipMalloc(&c->d_cout, co)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_cin, ci)) != hipSuccess || (e = hipHostMalloc(&c->h_cout, co)) != hipSuccess)
      return bail(DP_ENOMEM, "frame staging (device / pinned)", e);
    c->cin_cap = ci;
    c->cout_cap = co;
  }
  tr.mark("sums+alloc");
  par_for(c, T, [&](uint32_t t) {
    uint64_t p = acc[t];
    for (uint32_t i = (uint32_t)((uint64_t)n * t / T), b = (uint32_t)((uint64_t)n * (t + 1) / T); i < b; i++) {
      c->h_pos[i] = (uint32_t)p;
      c->h_in[i] = in[i];
      p += ((in[i].off + in[i].len + 15u) >> 4) - (in[i].off >> 4);
    }
  });
  // the frames of packets [a, b): host threads pack their spans
  // (DPGPU_HOST_PLAIN: plain memcpy both ways, the A/B of scripts/probe/host_ab.py)
  const bool plain = getenv("DPGPU_HOST_PLAIN") != nullptr;
  auto gather = [&](uint32_t a, uint32_t b) {
    par_for(c, T, [&](uint32_t t) {
      for (uint32_t i = a + (uint32_t)((uint64_t)(b - a) * t / T), e = a + (uint32_t)((uint64_t)(b - a) * (t + 1) / T);
           i < e; i++) {
        if (i + 8 < e) __builtin_prefetch(buf + (in[i + 8].off & ~15u));
        const uint64_t lo = in[i].off & ~15u, u = ((in[i].off + in[i].len + 15u) >> 4) - (in[i].off >> 4);
        uint8_t *dst = c->h_cin + 16ull * c->h_pos[i];
        // the rounded-up end may lie past the caller's buffer: never read there
        if (!plain && lo + 16 * u <= buf_bytes) put_span(dst, buf + lo, u);
        else memcpy(dst, buf + lo, std::min<uint64_t>(16 * u, buf_bytes - lo));
      }
      _mm_sfence();  // the streamed spans are visible before the copies are enqueued
    });
  };
  tr.mark("positions");
  const uint32_t nch = !c->ft ? std::max<uint32_t>(1, std::min<uint32_t>(n / kHostChunk, 256)) : 1;
  if (nch > 1 && !c->host_streams) {
    for (int k = 0; k < kHostStreams; k++)
      if ((e = hipStreamCreateWithFlags(&c->hs[k], hipStreamNonBlocking)) != hipSuccess)
        return bail(DP_EIO, "hipStreamCreate (host path)", e);
    for (auto &ev : c->hev)
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess)
        return bail(DP_EIO, "hipEventCreate (host path)", e);
    c->host_streams = true;
  }
  while (c->chunk_ev.size() < nch) {
    hipEvent_t ev = nullptr;
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bail(DP_EIO, "hipEventCreate (chunks)", e);
    c->chunk_ev.push_back(ev);
  }
  if (stats && (e = hipMemsetAsync(c->d_stats, 0, sizeof(uint64_t) * DP_DONE_COUNT, s)) != hipSuccess)
    return bail(DP_EIO, "memset stats", e);
  // every host stream starts after the context stream's prior work (and the
  // stats clear); the context stream then waits for all of them
  if (nch > 1) {
    if ((e = hipEventRecord(c->hev[kHostStreams], s)) != hipSuccess) return bail(DP_EIO, "event record", e);
    for (int k = 0; k < kHostStreams; k++)
      if ((e = hipStreamWaitEvent(c->hs[k], c->hev[kHostStreams], 0)) != hipSuccess) return bail(DP_EIO, "stream wait", e);
  }
  int rc = 0;
  auto chunk_of = [&](uint32_t k, uint32_t &first, uint32_t &cnt) {
    first = (uint32_t)((uint64_t)n * k / nch);
    cnt = (uint32_t)((uint64_t)n * (k + 1) / nch) - first;
  };
  // in phases of chunks: a phase's frames are packed while the previous
  // phases' copies and kernels run
  const uint32_t phases = std::min<uint32_t>(nch, 4);
  uint32_t gathered = 0;  // chunks whose frames are packed
  for (uint32_t k = 0; k < nch && !rc; k++) {
    uint32_t first, cnt;
    if (k == gathered) {  // phase ph holds chunks [nch * ph / phases, nch * (ph + 1) / phases)
      uint32_t ph = 0;
      while ((uint64_t)nch * (ph + 1) / phases <= k) ph++;
      const uint32_t k1 = (uint32_t)((uint64_t)nch * (ph + 1) / phases);
      gather((uint32_t)((uint64_t)n * k / nch), (uint32_t)((uint64_t)n * k1 / nch));
      gathered = k1;
    }
    chunk_of(k, first, cnt);
    hipStream_t hs = nch == 1 ? s : c->hs[k % kHostStreams];
    const uint64_t b0 = 16ull * c->h_pos[first], b1 = first + cnt < n ? 16ull * c->h_pos[first + cnt] : in_bytes;
    const uint64_t o0 = b0 + (uint64_t)grow * first, o1 = b1 + (uint64_t)grow * (first + cnt);
    if ((e = hipMemcpyAsync(c->d_cin + b0, c->h_cin + b0, b1 - b0, hipMemcpyHostToDevice, hs)) != hipSuccess ||
        (e = hipMemcpyAsync(c->d_pos + first, c->h_pos + first, sizeof(uint32_t) * cnt, hipMemcpyHostToDevice, hs)) != hipSuccess ||
        (e = hipMemcpyAsync(c->d_in + first, c->h_in + first, sizeof(dp_pkt_in_t) * cnt, hipMemcpyHostToDevice, hs)) != hipSuccess) {
      rc = fail(DP_EIO, "H2D chunk", e);
      break;
    }
    if (dpk_stage_expand(c->d_cin, c->d_pos + first, c->d_in + first, c->d_buf, cnt, hs)) { rc = fail(DP_EIO, "stage expand"); break; }
    if ((rc = dp_process_burst_device(c, c->d_buf, need, c->d_in + first, c->d_out + first, dm ? dm + first : nullptr,
                                      cnt, stats ? c->d_stats : nullptr, hs)))
      break;
    if (dpk_stage_collect(c->d_buf, c->d_pos + first, c->d_in + first, c->d_cout + (uint64_t)grow * first, grow, cnt, hs)) {
      rc = fail(DP_EIO, "stage collect");
      break;
    }
    if ((e = hipMemcpyAsync(c->h_cout + o0, c->d_cout + o0, o1 - o0, hipMemcpyDeviceToHost, hs)) != hipSuccess ||
        (e = hipMemcpyAsync(c->h_out + first, c->d_out + first, sizeof(dp_pkt_out_t) * cnt, hipMemcpyDeviceToHost, hs)) != hipSuccess ||
        (meta && (e = hipMemcpyAsync(c->h_meta + first, dm + first, sizeof(dp_pkt_meta_t) * cnt, hipMemcpyDeviceToHost, hs)) != hipSuccess) ||
        (e = hipEventRecord(c->chunk_ev[k], hs)) != hipSuccess) {
      rc = fail(DP_EIO, "D2H chunk", e);
      break;
    }
  }
  if (nch > 1) {
    for (int k = 0; k < kHostStreams; k++) {
      (void)hipEventRecord(c->hev[k], c->hs[k]);
      (void)hipStreamWaitEvent(s, c->hev[k], 0);
    }
  }
  if (rc) {
    (void)hipStreamSynchronize(s);
    mark_failed_host(in, out, meta, n);
    return rc;
  }
  // write-back as each chunk lands: records, and each delivered frame from
  // its packed span (an output outside its staged span -- a publish that
  // added encapsulation between this burst's staging and its launch -- is an
  // InternalFailure of that packet)
  tr.mark("gather+enqueue");
  // Work items of at most kWbItem packets, taken in chunk order by whichever
  // thread is free (a whole chunk per thread left the last chunks to a few
  // threads while the rest idled)
  std::atomic<int> werr{0};
  constexpr uint32_t kWbItem = 8192;
  std::vector<uint32_t> item0(nch + 1, 0);  // first work item of each chunk
  for (uint32_t k = 0; k < nch; k++) {
    uint32_t first, cnt;
    chunk_of(k, first, cnt);
    item0[k + 1] = item0[k] + (cnt + kWbItem - 1) / kWbItem;
  }
  std::atomic<uint32_t> next_item{0};
  std::vector<std::atomic<uint8_t>> landed(nch);
  for (auto &x : landed) x.store(0, std::memory_order_relaxed);
  par_for(c, T, [&](uint32_t) {
    (void)hipSetDevice(c->device);
    uint32_t k = 0;
    for (uint32_t it; (it = next_item.fetch_add(1, std::memory_order_relaxed)) < item0[nch];) {
      while (item0[k + 1] <= it) k++;
      if (!landed[k].load(std::memory_order_acquire)) {
        const hipError_t we = hipEventSynchronize(c->chunk_ev[k]);
        if (we != hipSuccess) { werr = (int)we; continue; }
        landed[k].store(1, std::memory_order_release);
      }
      uint32_t first, cnt;
      chunk_of(k, first, cnt);
      const uint32_t a = first + (it - item0[k]) * kWbItem, b = std::min(first + cnt, a + kWbItem);
      for (uint32_t i = a; i < b; i++) {
        if (i + 8 < b) __builtin_prefetch(buf + in[i + 8].off, 1);
        dp_pkt_out_t o = c->h_out[i];
        if (o.done == DP_DONE_DELIVERED) {
          const uint64_t lo = (uint64_t)(in[i].off & ~15u) - grow, hi = (in[i].off + in[i].len + 15u) & ~15u;
          if (o.off >= lo && (uint64_t)o.off + o.len <= hi && (uint64_t)o.off + o.len <= buf_bytes)
          {
            const uint8_t *src = c->h_cout + 16ull * c->h_pos[i] + (uint64_t)grow * i + (o.off - lo);
            if (plain) memcpy(buf + o.off, src, o.len);
            else put_frame(buf + o.off, src, o.len);
          }
          else
            o = dp_pkt_out_t{in[i].off, in[i].len, DP_DONE_INTERNAL_FAILURE};
        }
        out[i] = o;
        if (meta) meta[i] = c->h_meta[i];
      }
    }
  });
  tr.mark("wait+write-back");
  tr.done(n, T, nch);
  if (werr) {
    (void)hipStreamSynchronize(s);
    return bail(DP_EIO, "chunk completion", (hipError_t)werr.load());
  }
  uint64_t hstats[DP_DONE_COUNT];
  if (stats && (e = hipMemcpyAsync(hstats, c->d_stats, sizeof(hstats), hipMemcpyDeviceToHost, s)) != hipSuccess) return bail(DP_EIO, "D2H stats", e);
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return bail(DP_EIO, "stream sync", e);
  if (stats) for (int k = 0; k < DP_DONE_COUNT; k++) stats[k] += hstats[k];
  return 0;
}

int dp_process_burst_sharded(dp_ctx_t *const *ctxs, uint32_t n_ctx, uint8_t *buf, uint64_t buf_bytes,
                             const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n,
                             uint64_t *stats) {
  if (!ctxs || n_ctx == 0) { mark_failed_host(in, out, meta, n); return fail(DP_EINVAL, "no contexts"); }
  if (n == 0) return 0;
  if (!buf || !in || !out) { mark_failed_host(in, out, meta, n); return fail(DP_EINVAL, "null burst buffers"); }
  // packets in buffer order, each owning [off - DP_HEADROOM, off + len): the
  // shards' byte spans are then disjoint and can be copied back concurrently
  for (uint32_t i = 0; i < n; i++) {
    const bool inside = in[i].off >= DP_HEADROOM && (uint64_t)in[i].off + in[i].len <= buf_bytes;
    const bool ordered = i == 0 || in[i].off - DP_HEADROOM >= (uint64_t)in[i - 1].off + in[i - 1].len;
    if (!inside || !ordered) {
      mark_failed_host(in, out, meta, n);
      return fail(DP_EINVAL, "sharded bursts need in-order, non-overlapping packet slots");
    }
  }
  for (uint32_t k = 0; k < n_ctx; k++) {
    if (!ctxs[k]) { mark_failed_host(in, out, meta, n); return fail(DP_EINVAL, "null context"); }
    // With a flow table, every context shares it (the reference's one
    // Arc<FlowTable> behind every worker's pipeline, packet_processor/mod.rs:
    // 68,100-120): the shards are the workers' bursts, and the table's order
    // (its last_burst event, taken under its lock) runs their flows launches
    // one after the other in shard order -- one of the orders the reference's
    // concurrent workers may take.  A table lives on one device, so such
    // shards share it (contexts of one GPU); the copies still overlap.
    if (ctxs[k]->ft != ctxs[0]->ft) {
      mark_failed_host(in, out, meta, n);
      return fail(DP_EINVAL, "sharded bursts: every context attached to the same flow table, or none");
    }
  }
  struct Shard {
    uint32_t first, cnt;
    uint64_t lo, hi;               // byte span in `buf`
    std::vector<dp_pkt_in_t> rin;  // in-records rebased to the span
    uint64_t st[DP_DONE_COUNT];
  };
  std::vector<Shard> sh(n_ctx);
  int rc = 0;
  for (uint32_t k = 0; k < n_ctx; k++) {
    Shard &S = sh[k];
    S.first = (uint32_t)((uint64_t)n * k / n_ctx);
    S.cnt = (uint32_t)((uint64_t)n * (k + 1) / n_ctx) - S.first;
    if (!S.cnt) continue;
    // 64-byte aligned start, never below the previous packet's end: the
    // spans are disjoint, so the concurrent copies back never overlap
    const uint64_t prev_end = S.first ? (uint64_t)in[S.first - 1].off + in[S.first - 1].len : 0;
    S.lo = std::max<uint64_t>(prev_end, (in[S.first].off - DP_HEADROOM) & ~63ull);
    const dp_pkt_in_t &last = in[S.first + S.cnt - 1];
    S.hi = std::min<uint64_t>(buf_bytes, (uint64_t)last.off + last.len);
    S.rin.assign(in + S.first, in + S.first + S.cnt);
    for (auto &r : S.rin) r.off -= (uint32_t)S.lo;
  }
  // stage and launch every shard on its own device, then collect
  std::vector<int> launched(n_ctx, 0);
  for (uint32_t k = 0; k < n_ctx && !rc; k++) {
    Shard &S = sh[k];
    if (!S.cnt) continue;
    dp_ctx *c = ctxs[k];
    (void)hipSetDevice(c->device);
    const uint64_t bytes = S.hi - S.lo;
    const uint64_t need = ((bytes + 15) & ~15ull) + 16;
    hipError_t e = hipSuccess;
    if (need > c->d_buf_cap) {
      if (c->d_buf) { (void)hipStreamSynchronize(c->stream); (void)hipFree(c->d_buf); }
      c->d_buf = nullptr;
      c->d_buf_cap = 0;
      if ((e = hipMalloc(&c->d_buf, need)) != hipSuccess) { rc = fail(DP_ENOMEM, "hipMalloc shard", e); break; }
      c->d_buf_cap = need;
    }
    if ((e = ensure_records(c, S.cnt)) != hipSuccess) { rc = fail(DP_ENOMEM, "hipMalloc shard records", e); break; }
    hipStream_t s = c->stream;
    dp_pkt_meta_t *dm = meta ? c->d_meta : nullptr;
    if ((e = hipMemcpyAsync(c->d_buf, buf + S.lo, bytes, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(c->d_in, S.rin.data(), sizeof(dp_pkt_in_t) * S.cnt, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (stats && (e = hipMemsetAsync(c->d_stats, 0, sizeof(uint64_t) * DP_DONE_COUNT, s)) != hipSuccess)) {
      rc = fail(DP_EIO, "H2D shard", e);
      break;
    }
    if ((rc = dp_process_burst_device(c, c->d_buf, need, c->d_in, c->d_out, dm, S.cnt, stats ? c->d_stats : nullptr, s)))
      break;
    if ((e = hipMemcpyAsync(buf + S.lo, c->d_buf, bytes, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(out + S.first, c->d_out, sizeof(dp_pkt_out_t) * S.cnt, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (meta && (e = hipMemcpyAsync(meta + S.first, dm, sizeof(dp_pkt_meta_t) * S.cnt, hipMemcpyDeviceToHost, s)) != hipSuccess) ||
        (stats && (e = hipMemcpyAsync(S.st, c->d_stats, sizeof(S.st), hipMemcpyDeviceToHost, s)) != hipSuccess)) {
      rc = fail(DP_EIO, "D2H shard", e);
      break;
    }
    launched[k] = 1;
  }
  for (uint32_t k = 0; k < n_ctx; k++) {
    if (!launched[k]) continue;
    (void)hipSetDevice(ctxs[k]->device);
    hipError_t e = hipStreamSynchronize(ctxs[k]->stream);
    if (e != hipSuccess && !rc) rc = fail(DP_EIO, "shard stream sync", e);
  }
  if (rc) { mark_failed_host(in, out, meta, n); return rc; }
  for (uint32_t k = 0; k < n_ctx; k++) {
    Shard &S = sh[k];
    for (uint32_t i = 0; i < S.cnt; i++) out[S.first + i].off += (uint32_t)S.lo;
    if (stats && S.cnt)
      for (int r = 0; r < DP_DONE_COUNT; r++) stats[r] += S.st[r];
  }
  return 0;
}

int dp_ctx_synchronize(dp_ctx_t *c) {
  if (!c) return DP_EINVAL;
  hipError_t e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return fail(DP_EIO, "stream sync", e);
  reap(c);
  return 0;
}

// DPDK rx burst -> path -> tx-ready mbufs (include/dpgpu.h "DPDK rx / tx
// burst glue"): the frames stay in their mempool memory, the kernel works on
// them over PCIe (the zero-copy host path), only the records are the
// context's own pinned arrays.
int dp_process_mbufs(dp_ctx_t *c, const void *pool_base, uint64_t pool_bytes, void *const *mbufs, uint32_t n,
                     const dp_mbuf_layout_t *layout, const uint32_t *port_ifindex, uint32_t n_ports,
                     dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint64_t *stats) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!out || !mbufs || !layout || !pool_base) {
    mark_failed_host(nullptr, out, meta, n);
    return fail(DP_EINVAL, "null argument");
  }
  (void)hipSetDevice(c->device);
  if (n > c->mb_cap) {
    if (c->mb_in) (void)hipHostFree(c->mb_in);
    if (c->mb_out) (void)hipHostFree(c->mb_out);
    if (c->mb_meta) (void)hipHostFree(c->mb_meta);
    c->mb_in = nullptr;
    c->mb_out = nullptr;
    c->mb_meta = nullptr;
    c->mb_cap = 0;
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&c->mb_in), sizeof(dp_pkt_in_t) * n, hipHostMallocMapped);
    if (e == hipSuccess)
      e = hipHostMalloc(reinterpret_cast<void **>(&c->mb_out), sizeof(dp_pkt_out_t) * n, hipHostMallocMapped);
    if (e == hipSuccess)
      e = hipHostMalloc(reinterpret_cast<void **>(&c->mb_meta), sizeof(dp_pkt_meta_t) * n, hipHostMallocMapped);
    if (e != hipSuccess) {
      mark_failed_host(nullptr, out, meta, n);
      return fail(DP_ENOMEM, "pinned mbuf burst records", e);
    }
    c->mb_cap = n;
  }
  std::vector<dp_pkt_in_t> rin(n);
  int rc = dp_mbuf_burst_in(pool_base, pool_bytes, mbufs, n, layout, port_ifindex, n_ports, rin.data());
  if (rc) { mark_failed_host(nullptr, out, meta, n); return fail(rc, "mbuf burst records"); }
  // an mbuf outside the layout contract is InternalFailure on its own; the
  // others run as one burst
  std::vector<uint32_t> idx;
  idx.reserve(n);
  for (uint32_t i = 0; i < n; i++)
    if (rin[i].off >= DP_HEADROOM) { c->mb_in[idx.size()] = rin[i]; idx.push_back(i); }
  mark_failed_host(rin.data(), out, meta, n);
  const int mode = c->host_path;
  c->host_path = DP_HOST_ZERO_COPY;
  rc = idx.empty() ? 0 : dp_process_burst(c, const_cast<uint8_t *>(static_cast<const uint8_t *>(pool_base)),
                                          pool_bytes, c->mb_in, c->mb_out, meta ? c->mb_meta : nullptr,
                                          (uint32_t)idx.size(), stats);
  c->host_path = mode;
  if (rc) return rc;  // every out[i] InternalFailure
  for (size_t j = 0; j < idx.size(); j++) {
    out[idx[j]] = c->mb_out[j];
    if (meta) meta[idx[j]] = c->mb_meta[j];
  }
  if (stats) stats[DP_DONE_INTERNAL_FAILURE] += n - idx.size();
  rc = dp_mbuf_burst_out(mbufs, n, layout, rin.data(), out);
  return rc ? fail(rc, "mbuf burst results") : 0;
}

}  // extern "C"

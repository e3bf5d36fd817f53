// SPDX-License-Identifier: Apache-2.0
//
// Flow table API (include/dpgpu.h "Flow table"): FlowTable
// (flow-entry/src/flow_table/table.rs:24-330) as an HBM open-addressing
// table of 128-byte slots (dp_flow.h).  Every operation is a batch kernel on
// the table's own stream; the order-dependent decisions of a batch of inserts
// (capacity, replacement) are taken on the host between a probe kernel and a
// claim kernel, so a batch behaves exactly like the reference's inserts one
// after the other.  Bursts read the table concurrently: a slot is filled
// behind a BUSY state and published with a release store of FULL, so a burst
// sees a flow either whole or not at all; a burst launched after an insert
// call returns sees it.
#include <hip/hip_runtime.h>

#include <cstring>
#include <unordered_set>
#include <string>
#include <vector>

#include "../../include/dpgpu.h"
#include "dp_flows_rt.h"

using dpf::FlowSlot;
using dpf::FKey;

namespace {

constexpr uint32_t kTB = 256;

// FlowTable::lookup by key: linear probing from the key's home slot, at most
// max_probe + 1 slots (no stored flow sits further from its home)
__device__ __forceinline__ uint32_t probe(const FlowSlot *slots, uint32_t mask, uint32_t max_probe, const FKey &k,
                                          uint32_t &state) {
  uint32_t i = dpf::fkey_hash(k) & mask;
  for (uint32_t p = 0; p <= max_probe; p++) {
    const FlowSlot &s = slots[i];
    const uint32_t st = __hip_atomic_load(&s.state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if ((st & 3u) == dpf::FS_EMPTY) return dpf::kNoSlot;
    if ((st & 3u) == dpf::FS_FULL && s.src_vni == k.w[0] && s.fk == k.w[1] && s.ports == k.w[2] &&
        s.src[0] == k.w[3] && s.src[1] == k.w[4] && s.src[2] == k.w[5] && s.src[3] == k.w[6] &&
        s.dst[0] == k.w[7] && s.dst[1] == k.w[8] && s.dst[2] == k.w[9] && s.dst[3] == k.w[10]) {
      state = st;
      return i;
    }
    i = (i + 1) & mask;
  }
  return dpf::kNoSlot;
}

__device__ __forceinline__ bool ref_live(const FlowSlot *slots, uint32_t mask, uint64_t ref) {
  const uint32_t sl = (uint32_t)ref;
  return ref != ~0ull && sl <= mask && slots[sl].state == ((uint32_t)(ref >> 32) << 2 | dpf::FS_FULL);
}

__device__ void fill_info(const FlowSlot *slots, uint32_t mask, uint32_t sl, dp_flow_info_t &o) {
  const FlowSlot &s = slots[sl];
  o.ref = dpf::make_ref(sl, s.state);
  o.status = s.status;
  o.flags = s.flags;
  o.dst_vni = s.dst_vni;
  o.pad = 0;
  o.genid = s.genid;
  o.expires_at = s.expires_at;
  o.related = DP_FLOW_NONE;
  if (s.related <= mask && slots[s.related].state == s.related_tag)
    o.related = dpf::make_ref(s.related, s.related_tag);
  o.flags = s.flags & 7u;
  if (s.flags & dpf::kFlagPf) {  // PortFwState (nat/src/portfw/flow_state.rs:29-35)
    o.pf = (uint8_t)(s.pf & 0xffu);
    o.pf_status = (uint8_t)((s.pf >> 8) & 0xffu);
    o.pf_port = (uint16_t)(s.pf >> 16);
    o.pf_rule = s.pf_rule;
    o.pf_family = (uint8_t)s.pf_fam;
    for (int j = 0; j < 4; j++)
      for (int b = 0; b < 4; b++) o.pf_ip[4 * j + b] = (uint8_t)(s.pf_ip[j] >> (24 - 8 * b));
  }
}

__global__ void __launch_bounds__(kTB) fl_find_k(const FlowSlot *slots, uint32_t mask, uint32_t max_probe,
                                                const FKey *keys, uint32_t n, uint32_t *slot_out) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  uint32_t st;
  slot_out[i] = probe(slots, mask, max_probe, keys[i], st);
}

struct InsRec {
  FKey k;
  uint32_t slot;        // the slot of the flow this one replaces, kNoSlot: a new slot
  uint32_t flags, dst_vni;
  int64_t genid;
  uint64_t expires_at;
};

// Fill one slot per record: the replaced flow's slot, or the first EMPTY /
// TOMB slot of the key's probe sequence (claimed by CAS).  The new FlowInfo
// is Active (table.rs:235-240), with no related flow yet.  A new slot's
// displacement from the key's home raises the table's probe bound (*meta).
__global__ void __launch_bounds__(kTB) fl_insert_k(FlowSlot *slots, uint32_t mask, const InsRec *recs, uint32_t n,
                                                  uint64_t *refs, uint32_t *meta) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  const InsRec r = recs[i];
  uint32_t sl = r.slot, old = 0;
  if (sl != dpf::kNoSlot) {
    old = slots[sl].state;
    atomicExch(&slots[sl].state, (old & ~3u) | dpf::FS_BUSY);
  } else {
    uint32_t p = dpf::fkey_hash(r.k) & mask;
    for (uint32_t tries = 0; tries <= 2 * mask + 1; tries++) {
      old = __hip_atomic_load(&slots[p].state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t st = old & 3u;
      if ((st == dpf::FS_EMPTY || st == dpf::FS_TOMB) &&
          atomicCAS(&slots[p].state, old, (old & ~3u) | dpf::FS_BUSY) == old) {
        sl = p;
        atomicMax(meta, (p - (dpf::fkey_hash(r.k) & mask)) & mask);
        break;
      }
      if (st == dpf::FS_FULL || st == dpf::FS_BUSY) p = (p + 1) & mask;
    }
    if (sl == dpf::kNoSlot) { refs[i] = ~0ull; return; }
  }
  FlowSlot &s = slots[sl];
  s.src_vni = r.k.w[0]; s.fk = r.k.w[1]; s.ports = r.k.w[2];
  for (int j = 0; j < 4; j++) { s.src[j] = r.k.w[3 + j]; s.dst[j] = r.k.w[7 + j]; }
  s.status = DP_FLOW_ACTIVE;
  s.flags = r.flags;
  s.dst_vni = r.dst_vni;
  s.related = dpf::kNoSlot;
  s.related_tag = 0;
  s.mark = dpf::kIdleMark;
  s.genid = r.genid;
  s.expires_at = r.expires_at;
  s.pf = 0;
  s.pf_rule = 0;
  const uint32_t tag = ((old >> 2) + 1) & 0x3fffffffu;
  const uint32_t st = (tag << 2) | dpf::FS_FULL;
  __hip_atomic_store(&s.state, st, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  refs[i] = dpf::make_ref(sl, st);
}

// related_pair: each flow's Weak to the other (flow_info.rs:290-339)
__global__ void fl_link_k(FlowSlot *slots, uint32_t mask, uint64_t a, uint64_t b) {
  const uint32_t sa = (uint32_t)a, sb = (uint32_t)b;
  if (!ref_live(slots, mask, a) || !ref_live(slots, mask, b)) return;
  slots[sa].related = sb;
  slots[sa].related_tag = slots[sb].state;
  slots[sb].related = sa;
  slots[sb].related_tag = slots[sa].state;
}

__global__ void __launch_bounds__(kTB) fl_lookup_k(const FlowSlot *slots, uint32_t mask, uint32_t max_probe,
                                                  const FKey *keys, uint32_t n, dp_flow_info_t *out) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  uint32_t st;
  const uint32_t sl = probe(slots, mask, max_probe, keys[i], st);
  dp_flow_info_t o{};
  o.ref = DP_FLOW_NONE;
  o.related = DP_FLOW_NONE;
  if (sl != dpf::kNoSlot) fill_info(slots, mask, sl, o);
  out[i] = o;
}

__global__ void __launch_bounds__(kTB) fl_get_k(const FlowSlot *slots, uint32_t mask, const uint64_t *refs, uint32_t n,
                                               dp_flow_info_t *out) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  dp_flow_info_t o{};
  o.ref = DP_FLOW_NONE;
  o.related = DP_FLOW_NONE;
  if (ref_live(slots, mask, refs[i])) fill_info(slots, mask, (uint32_t)refs[i], o);
  out[i] = o;
}

// FlowTable::remove (table.rs:282-295): Detached, out of the table
__global__ void __launch_bounds__(kTB) fl_remove_k(FlowSlot *slots, uint32_t mask, uint32_t max_probe,
                                                  const FKey *keys, uint32_t n, uint32_t *count) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  uint32_t st;
  const uint32_t sl = probe(slots, mask, max_probe, keys[i], st);
  if (sl == dpf::kNoSlot) return;
  slots[sl].status = DP_FLOW_DETACHED;
  if (atomicCAS(&slots[sl].state, st, (st & ~3u) | dpf::FS_TOMB) != st) return;
  atomicAdd(count, 1u);
  // the new tombstone ends a cluster: it and the tombstones before it
  // become EMPTY (as fl_reclaim_k; a missed reclaim only costs probe length)
  if ((__hip_atomic_load(&slots[(sl + 1) & mask].state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) & 3u) !=
      dpf::FS_EMPTY)
    return;
  uint32_t j = sl;
  for (uint32_t k = 0; k < mask; k++, j = (j - 1) & mask) {
    const uint32_t o = __hip_atomic_load(&slots[j].state, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if ((o & 3u) != dpf::FS_TOMB) break;
    atomicCAS(&slots[j].state, o, (o & ~3u) | dpf::FS_EMPTY);
  }
}

// FlowInfo::invalidate_pair (flow_info.rs:449-455)
__global__ void __launch_bounds__(kTB) fl_invalidate_k(FlowSlot *slots, uint32_t mask, const uint64_t *refs, uint32_t n) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n || !ref_live(slots, mask, refs[i])) return;
  FlowSlot &s = slots[(uint32_t)refs[i]];
  s.status = DP_FLOW_CANCELLED;
  if (s.related <= mask && slots[s.related].state == s.related_tag) slots[s.related].status = DP_FLOW_CANCELLED;
}

__global__ void fl_set_status_k(FlowSlot *slots, uint32_t mask, uint64_t ref, uint32_t status, uint32_t *ok) {
  *ok = 0;
  if (!ref_live(slots, mask, ref)) return;
  slots[(uint32_t)ref].status = status;
  *ok = 1;
}

// The flow timers up to `now` (FlowTable::start_timer, table.rs:160-213)
__global__ void __launch_bounds__(kTB) fl_sweep_k(FlowSlot *slots, uint64_t nslots, uint64_t now,
                                                 unsigned long long *count) {
  for (uint64_t i = blockIdx.x * (uint64_t)kTB + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * kTB) {
    FlowSlot &s = slots[i];
    const uint32_t st = s.state;
    if ((st & 3u) != dpf::FS_FULL) continue;
    bool gone = false;
    if (s.status == DP_FLOW_ACTIVE) {
      if (s.expires_at <= now) { s.status = DP_FLOW_EXPIRED; gone = true; }
    } else if (s.status == DP_FLOW_CANCELLED || s.status == DP_FLOW_EXPIRED) {
      gone = true;
    }
    if (gone && atomicCAS(&s.state, st, (st & ~3u) | dpf::FS_TOMB) == st) atomicAdd(count, 1ull);
  }
}

// Tombstone reclamation after removals: a run of TOMB slots that ends at an
// EMPTY slot becomes EMPTY (a probe passing through the run would stop at
// that EMPTY slot anyway, so every lookup's outcome is unchanged).  Each
// EMPTY slot's thread walks back over its own run; runs are disjoint.  Stored
// flows never move, so refs and related links stay valid; the fill tag is
// kept, so the next fill of a reclaimed slot still gets a new tag.
__global__ void __launch_bounds__(kTB) fl_reclaim_k(FlowSlot *slots, uint64_t nslots, unsigned long long *count) {
  const uint32_t mask = (uint32_t)(nslots - 1);
  for (uint64_t i = blockIdx.x * (uint64_t)kTB + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * kTB) {
    if ((slots[i].state & 3u) != dpf::FS_EMPTY) continue;
    uint32_t j = ((uint32_t)i - 1) & mask;
    unsigned long long c = 0;
    for (uint32_t k = 0; k < mask && j != (uint32_t)i; k++, j = (j - 1) & mask) {
      const uint32_t st = slots[j].state;
      if ((st & 3u) != dpf::FS_TOMB) break;
      slots[j].state = (st & ~3u) | dpf::FS_EMPTY;
      c++;
    }
    if (c) atomicAdd(count, c);
  }
}

// Slot census for dpf_debug_table_stats: FULL, TOMB, EMPTY
__global__ void __launch_bounds__(kTB) fl_census_k(const FlowSlot *slots, uint64_t nslots, unsigned long long *out) {
  unsigned long long c[3] = {0, 0, 0};
  for (uint64_t i = blockIdx.x * (uint64_t)kTB + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * kTB) {
    const uint32_t st = slots[i].state & 3u;
    c[0] += st == dpf::FS_FULL;
    c[1] += st == dpf::FS_TOMB;
    c[2] += st == dpf::FS_EMPTY;
  }
  for (int k = 0; k < 3; k++)
    if (c[k]) atomicAdd(&out[k], c[k]);
}

__global__ void __launch_bounds__(kTB) fl_count_k(const FlowSlot *slots, uint64_t nslots, unsigned long long *out) {
  unsigned long long len = 0, act = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)kTB + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * kTB) {
    if ((slots[i].state & 3u) != dpf::FS_FULL) continue;
    len++;
    act += slots[i].status == DP_FLOW_ACTIVE;
  }
  for (int o = 32; o > 0; o >>= 1) {
    len += __shfl_xor(len, o);
    act += __shfl_xor(act, o);
  }
  if ((threadIdx.x & 63) == 0 && (len | act)) {
    atomicAdd(&out[0], len);
    atomicAdd(&out[1], act);
  }
}

// --------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------
FKey key_words(const dp_flow_key_t &x) {
  FKey k{};
  k.w[0] = x.src_vni;
  k.w[1] = (uint32_t)x.family | ((uint32_t)x.kind << 8);
  k.w[2] = ((uint32_t)x.sport << 16) | x.dport;
  uint8_t s[16] = {0}, d[16] = {0};
  const size_t n = x.family == 4 ? 4 : 16;
  memcpy(s, x.src, n);
  memcpy(d, x.dst, n);
  memcpy(&k.w[3], s, 16);
  memcpy(&k.w[7], d, 16);
  return k;
}

// What a FlowInfo can hold here (same checks as the oracle's flow_check).
bool flow_valid(const dp_flow_t &f) {
  const dp_flow_key_t &x = f.key;
  if (x.family != 4 && x.family != 6) return false;
  if (x.kind < DP_FLOW_TCP || x.kind > DP_FLOW_ICMP_OTHER) return false;
  if ((x.kind == DP_FLOW_TCP || x.kind == DP_FLOW_UDP) && (x.sport == 0 || x.dport == 0)) return false;
  if (x.kind == DP_FLOW_ICMP_QUERY && x.dport) return false;
  if (x.kind == DP_FLOW_ICMP_OTHER && (x.sport || x.dport)) return false;
  if (x.src_vni >= (1u << 24) || f.dst_vni == 0 || f.dst_vni >= (1u << 24)) return false;
  if (f.flags & ~7u) return false;
  return true;
}

using Scratch = FlowScratch;

// Run `f(stream)` with the table's device current and its stream; sync.
template <class F>
int run(dp_flow_table *ft, const char *what, F f) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(ft->device);
  // after every flows burst launched before this call (dp_flows_rt.h)
  if (ft->burst_armed) (void)hipStreamWaitEvent(ft->stream, ft->last_burst, 0);
  int rc = f(ft->stream);
  hipError_t e = hipStreamSynchronize(ft->stream);
  if (!rc && e != hipSuccess) rc = dpr_fail(DP_EIO, what, e);
  if (!rc && (e = hipGetLastError()) != hipSuccess) rc = dpr_fail(DP_EIO, what, e);
  (void)hipSetDevice(prev);
  return rc;
}

uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kTB - 1) / kTB); }

// The table's device words ([0] probe bound, [2..3] len): bursts that create
// flows (port forwarding) move them on the device, so a management call that
// decides on the host reads them first and writes them back after.
int pull_meta(dp_flow_table *ft) {
  uint32_t m[4] = {0, 0, 0, 0};
  int rc = run(ft, "flow table counters", [&](hipStream_t st) {
    if (hipMemcpyAsync(m, ft->d_meta, sizeof(m), hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow table counters copy");
    return 0;
  });
  if (rc) return rc;
  ft->max_probe = m[0];
  ft->len = ((uint64_t)m[3] << 32) | m[2];
  return 0;
}
int push_meta(dp_flow_table *ft) {
  const uint32_t m[4] = {ft->max_probe, 0, (uint32_t)ft->len, (uint32_t)(ft->len >> 32)};
  return run(ft, "flow table counters", [&](hipStream_t st) {
    if (hipMemcpyAsync(ft->d_meta, m, sizeof(m), hipMemcpyHostToDevice, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow table counters copy");
    return 0;
  });
}

// Upload a host array into scratch `s`, returning its device copy.
template <class T>
T *upload(Scratch &s, const T *host, size_t n, hipStream_t st) {
  T *d = static_cast<T *>(s.get(sizeof(T) * (n ? n : 1)));
  if (!d) return nullptr;
  if (n && hipMemcpyAsync(d, host, sizeof(T) * n, hipMemcpyHostToDevice, st) != hipSuccess) return nullptr;
  return d;
}

// Sequential inserts of one batch of distinct keys (table.rs:215-260).
// `partner[i]`: index in the batch of the pair's first half whose activity
// admits flow i at capacity, or -1.
int insert_batch(dp_flow_table *ft, const dp_flow_t *flows, uint32_t n, const int32_t *partner,
                 uint64_t *refs, int32_t *results) {
  Scratch &s_keys = ft->scr[0], &s_slots = ft->scr[1], &s_recs = ft->scr[2], &s_refs = ft->scr[3];
  std::vector<FKey> keys(n);
  for (uint32_t i = 0; i < n; i++) keys[i] = key_words(flows[i].key);
  std::vector<uint32_t> found(n);
  int rc = run(ft, "flow probe", [&](hipStream_t st) {
    FKey *dk = upload(s_keys, keys.data(), n, st);
    uint32_t *ds = static_cast<uint32_t *>(s_slots.get(sizeof(uint32_t) * n));
    if (!dk || !ds) return dpr_fail(DP_ENOMEM, "flow scratch");
    hipLaunchKernelGGL(fl_find_k, dim3(blocks_for(n)), dim3(kTB), 0, st, ft->slots, ft->mask, ft->max_probe, dk, n,
                       ds);
    if (hipMemcpyAsync(found.data(), ds, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow probe copy");
    return 0;
  });
  if (rc) return rc;
  // the table never fills beyond 7/8 of its slots, so a free slot is always
  // within reach of a probe sequence
  const uint64_t hard = ft->nslots - ft->nslots / 8;
  std::vector<InsRec> recs;
  std::vector<uint32_t> which;
  std::vector<int32_t> res(n, DP_EFLOWCAP);
  std::vector<bool> accepted(n, false);
  uint64_t len = ft->len;
  for (uint32_t i = 0; i < n; i++) {
    const bool exception = partner[i] >= 0 && accepted[partner[i]];
    const bool is_new = found[i] == dpf::kNoSlot;
    if ((len >= ft->capacity && !exception) || (is_new && len >= hard)) continue;
    accepted[i] = true;
    res[i] = is_new ? DP_FLOW_INSERTED : DP_FLOW_REPLACED;
    if (is_new) len++;
    InsRec r{};
    r.k = keys[i];
    r.slot = found[i];
    r.flags = flows[i].flags;
    r.dst_vni = flows[i].dst_vni;
    r.genid = flows[i].genid;
    r.expires_at = flows[i].expires_at;
    recs.push_back(r);
    which.push_back(i);
  }
  std::vector<uint64_t> got(recs.size());
  uint32_t maxp = ft->max_probe;
  if (!recs.empty()) {
    rc = run(ft, "flow insert", [&](hipStream_t st) {
      InsRec *dr = upload(s_recs, recs.data(), recs.size(), st);
      uint64_t *df = static_cast<uint64_t *>(s_refs.get(sizeof(uint64_t) * recs.size()));
      if (!dr || !df) return dpr_fail(DP_ENOMEM, "flow scratch");
      hipLaunchKernelGGL(fl_insert_k, dim3(blocks_for(recs.size())), dim3(kTB), 0, st, ft->slots, ft->mask, dr,
                         (uint32_t)recs.size(), df, ft->d_meta);
      if (hipMemcpyAsync(got.data(), df, sizeof(uint64_t) * recs.size(), hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipMemcpyAsync(&maxp, ft->d_meta, sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess)
        return dpr_fail(DP_EIO, "flow insert copy");
      return 0;
    });
    if (rc) return rc;
  }
  // the probe bound covers every slot filled, whatever happens below
  ft->max_probe = maxp;
  // a flow that found no slot was never stored: the count takes only the
  // stored ones, then the whole batch reports the failure
  uint64_t lost = 0;
  for (size_t j = 0; j < recs.size(); j++)
    if (got[j] == ~0ull && recs[j].slot == dpf::kNoSlot) lost++;
  ft->len = len - lost;
  for (uint32_t i = 0; i < n; i++) {
    if (refs) refs[i] = DP_FLOW_NONE;
    if (results) results[i] = res[i];
  }
  for (size_t j = 0; j < recs.size(); j++) {
    if (got[j] == ~0ull) return dpr_fail(DP_EIO, "flow table probe exhausted");
    if (refs) refs[which[j]] = got[j];
  }
  return 0;
}

}  // namespace

extern "C" {

int dp_flow_table_create(int device_ordinal, uint64_t slots, dp_flow_table_t **out) {
  if (!out) return dpr_fail(DP_EINVAL, "null out");
  if (slots < 64 || (slots & (slots - 1)) || slots > (1ull << 31)) return dpr_fail(DP_EINVAL, "slots: a power of two in [64, 2^31]");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return dpr_fail(DP_ENODEV, "no HIP device", e);
  if (device_ordinal < 0 || device_ordinal >= ndev) return dpr_fail(DP_ENODEV, "bad device ordinal");
  dp_flow_table *ft = new dp_flow_table();
  ft->device = device_ordinal;
  ft->nslots = slots;
  ft->mask = (uint32_t)(slots - 1);
  ft->capacity = 10000000ull < slots / 2 ? 10000000ull : slots / 2;  // FlowTable::DEFAULT_CAPACITY
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device_ordinal);
  e = hipStreamCreateWithFlags(&ft->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ft->last_burst, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(&ft->slots, slots * sizeof(FlowSlot));
  if (e == hipSuccess) e = hipMalloc(&ft->d_meta, sizeof(uint32_t) * 4);
  if (e == hipSuccess) e = hipMemset(ft->d_meta, 0, sizeof(uint32_t) * 4);
  // every slot EMPTY with tag 0; marks idle
  if (e == hipSuccess) e = hipMemset(ft->slots, 0, slots * sizeof(FlowSlot));
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    if (ft->slots) (void)hipFree(ft->slots);
    if (ft->d_meta) (void)hipFree(ft->d_meta);
    if (ft->last_burst) (void)hipEventDestroy(ft->last_burst);
    if (ft->stream) (void)hipStreamDestroy(ft->stream);
    delete ft;
    return dpr_fail(DP_ENOMEM, "flow table allocation", e);
  }
  *out = ft;
  return 0;
}

int dp_flow_table_destroy(dp_flow_table_t *ft) {
  if (!ft) return DP_EINVAL;
  (void)hipSetDevice(ft->device);
  if (ft->burst_armed) (void)hipEventSynchronize(ft->last_burst);
  (void)hipStreamSynchronize(ft->stream);
  (void)hipFree(ft->slots);
  (void)hipFree(ft->d_meta);
  for (auto &x : ft->scr) x.release();
  (void)hipEventDestroy(ft->last_burst);
  (void)hipStreamDestroy(ft->stream);
  delete ft;
  return 0;
}

// Test hook (not part of dpgpu.h): out[0..3] = FULL, TOMB and EMPTY slots,
// and the table's probe bound (max_probe).
int dpf_debug_table_stats(dp_flow_table_t *ft, uint64_t *out) {
  if (!ft || !out) return dpr_fail(DP_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(ft->mu);
  Scratch &sc = ft->scr[0];
  unsigned long long c[3] = {0, 0, 0};
  int rc = run(ft, "flow census", [&](hipStream_t st) {
    unsigned long long *dc = static_cast<unsigned long long *>(sc.get(sizeof(c)));
    if (!dc) return dpr_fail(DP_ENOMEM, "flow scratch");
    if (hipMemsetAsync(dc, 0, sizeof(c), st) != hipSuccess) return dpr_fail(DP_EIO, "memset");
    const uint32_t b = blocks_for(ft->nslots) < 4096 ? blocks_for(ft->nslots) : 4096;
    hipLaunchKernelGGL(fl_census_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, dc);
    if (hipMemcpyAsync(c, dc, sizeof(c), hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow census copy");
    return 0;
  });
  if (rc) return rc;
  if (int rc2 = pull_meta(ft)) return rc2;
  out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = ft->max_probe;
  return 0;
}

int dp_flow_table_set_capacity(dp_flow_table_t *ft, uint64_t capacity) {
  if (!ft) return dpr_fail(DP_EINVAL, "null table");
  std::lock_guard<std::mutex> lk(ft->mu);
  ft->capacity = capacity;
  return 0;
}

int dp_flow_insert(dp_flow_table_t *ft, const dp_flow_t *flows, uint32_t n, uint64_t *refs, int32_t *results) {
  if (!ft || (!flows && n)) return dpr_fail(DP_EINVAL, "null argument");
  for (uint32_t i = 0; i < n; i++)
    if (!flow_valid(flows[i])) return dpr_fail(DP_EINVAL, "invalid flow");
  std::lock_guard<std::mutex> lk(ft->mu);
  if (int rc = pull_meta(ft)) return rc;
  // a key repeated within the batch splits it: each part holds distinct keys
  uint32_t s = 0;
  while (s < n) {
    std::unordered_set<std::string> seen;
    uint32_t e = s;
    for (; e < n; e++) {
      const FKey k = key_words(flows[e].key);
      if (!seen.insert(std::string(reinterpret_cast<const char *>(&k), sizeof(k))).second) break;
    }
    std::vector<int32_t> partner(e - s, -1);
    int rc = insert_batch(ft, flows + s, e - s, partner.data(), refs ? refs + s : nullptr,
                          results ? results + s : nullptr);
    if (rc) { (void)push_meta(ft); return rc; }
    s = e;
  }
  return push_meta(ft);
}

int dp_flow_insert_pair(dp_flow_table_t *ft, const dp_flow_t *a, const dp_flow_t *b, uint64_t *refs,
                        int32_t *results) {
  if (!ft || !a || !b) return dpr_fail(DP_EINVAL, "null argument");
  if (!flow_valid(*a) || !flow_valid(*b)) return dpr_fail(DP_EINVAL, "invalid flow");
  const FKey ka = key_words(a->key), kb = key_words(b->key);
  if (memcmp(&ka, &kb, sizeof(FKey)) == 0) return dpr_fail(DP_EINVAL, "a pair of identical keys");
  if (((a->flags ^ b->flags) & DP_FLOW_INITIATOR) == 0) return dpr_fail(DP_EINVAL, "exactly one initiator");
  std::lock_guard<std::mutex> lk(ft->mu);
  if (int rc = pull_meta(ft)) return rc;
  dp_flow_t both[2] = {*a, *b};
  const int32_t partner[2] = {-1, 0};
  uint64_t r[2];
  int32_t res[2];
  int rc = insert_batch(ft, both, 2, partner, r, res);
  if (int rc2 = push_meta(ft)) rc = rc ? rc : rc2;
  if (rc) return rc;
  if (r[0] != DP_FLOW_NONE && r[1] != DP_FLOW_NONE) {
    rc = run(ft, "flow link", [&](hipStream_t st) {
      hipLaunchKernelGGL(fl_link_k, dim3(1), dim3(1), 0, st, ft->slots, ft->mask, r[0], r[1]);
      return 0;
    });
    if (rc) return rc;
  }
  if (refs) { refs[0] = r[0]; refs[1] = r[1]; }
  if (results) { results[0] = res[0]; results[1] = res[1]; }
  return 0;
}

int dp_flow_lookup(dp_flow_table_t *ft, const dp_flow_key_t *keys, uint32_t n, dp_flow_info_t *out) {
  if (!ft || ((!keys || !out) && n)) return dpr_fail(DP_EINVAL, "null argument");
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(ft->mu);
  if (int rc = pull_meta(ft)) return rc;
  std::vector<FKey> k(n);
  for (uint32_t i = 0; i < n; i++) k[i] = key_words(keys[i]);
  Scratch &sk = ft->scr[0], &so = ft->scr[1];
  return run(ft, "flow lookup", [&](hipStream_t st) {
    FKey *dk = upload(sk, k.data(), n, st);
    dp_flow_info_t *d = static_cast<dp_flow_info_t *>(so.get(sizeof(dp_flow_info_t) * n));
    if (!dk || !d) return dpr_fail(DP_ENOMEM, "flow scratch");
    hipLaunchKernelGGL(fl_lookup_k, dim3(blocks_for(n)), dim3(kTB), 0, st, ft->slots, ft->mask, ft->max_probe, dk,
                       n, d);
    if (hipMemcpyAsync(out, d, sizeof(dp_flow_info_t) * n, hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow lookup copy");
    return 0;
  });
}

int dp_flow_get(dp_flow_table_t *ft, const uint64_t *refs, uint32_t n, dp_flow_info_t *out) {
  if (!ft || ((!refs || !out) && n)) return dpr_fail(DP_EINVAL, "null argument");
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(ft->mu);
  Scratch &sr = ft->scr[0], &so = ft->scr[1];
  return run(ft, "flow get", [&](hipStream_t st) {
    uint64_t *dr = upload(sr, refs, n, st);
    dp_flow_info_t *d = static_cast<dp_flow_info_t *>(so.get(sizeof(dp_flow_info_t) * n));
    if (!dr || !d) return dpr_fail(DP_ENOMEM, "flow scratch");
    hipLaunchKernelGGL(fl_get_k, dim3(blocks_for(n)), dim3(kTB), 0, st, ft->slots, ft->mask, dr, n, d);
    if (hipMemcpyAsync(out, d, sizeof(dp_flow_info_t) * n, hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow get copy");
    return 0;
  });
}

int dp_flow_remove(dp_flow_table_t *ft, const dp_flow_key_t *keys, uint32_t n, uint32_t *n_removed) {
  if (!ft || (!keys && n)) return dpr_fail(DP_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(ft->mu);
  if (int rc = pull_meta(ft)) return rc;
  std::vector<FKey> k(n ? n : 1);
  for (uint32_t i = 0; i < n; i++) k[i] = key_words(keys[i]);
  Scratch &sk = ft->scr[0], &sc = ft->scr[1];
  uint32_t cnt = 0;
  int rc = run(ft, "flow remove", [&](hipStream_t st) {
    FKey *dk = upload(sk, k.data(), n, st);
    uint32_t *dc = static_cast<uint32_t *>(sc.get(sizeof(uint32_t)));
    if (!dk || !dc) return dpr_fail(DP_ENOMEM, "flow scratch");
    if (hipMemsetAsync(dc, 0, sizeof(uint32_t), st) != hipSuccess) return dpr_fail(DP_EIO, "memset");
    if (n)
      hipLaunchKernelGGL(fl_remove_k, dim3(blocks_for(n)), dim3(kTB), 0, st, ft->slots, ft->mask, ft->max_probe,
                         dk, n, dc);
    if (hipMemcpyAsync(&cnt, dc, sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow remove copy");
    return 0;
  });
  if (rc) return rc;
  ft->len -= cnt;
  if (n_removed) *n_removed = cnt;
  return push_meta(ft);
}

int dp_flow_invalidate(dp_flow_table_t *ft, const uint64_t *refs, uint32_t n) {
  if (!ft || (!refs && n)) return dpr_fail(DP_EINVAL, "null argument");
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(ft->mu);
  Scratch &sr = ft->scr[0];
  return run(ft, "flow invalidate", [&](hipStream_t st) {
    uint64_t *dr = upload(sr, refs, n, st);
    if (!dr) return dpr_fail(DP_ENOMEM, "flow scratch");
    hipLaunchKernelGGL(fl_invalidate_k, dim3(blocks_for(n)), dim3(kTB), 0, st, ft->slots, ft->mask, dr, n);
    return 0;
  });
}

int dp_flow_set_status(dp_flow_table_t *ft, uint64_t ref, uint32_t status) {
  if (!ft || status > DP_FLOW_DETACHED) return dpr_fail(DP_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(ft->mu);
  Scratch &so = ft->scr[0];
  uint32_t ok = 0;
  int rc = run(ft, "flow set status", [&](hipStream_t st) {
    uint32_t *d = static_cast<uint32_t *>(so.get(sizeof(uint32_t)));
    if (!d) return dpr_fail(DP_ENOMEM, "flow scratch");
    hipLaunchKernelGGL(fl_set_status_k, dim3(1), dim3(1), 0, st, ft->slots, ft->mask, ref, status, d);
    if (hipMemcpyAsync(&ok, d, sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow set status copy");
    return 0;
  });
  if (rc) return rc;
  return ok ? 0 : dpr_fail(DP_EINVAL, "ref names no stored flow");
}

int dp_flow_sweep(dp_flow_table_t *ft, uint64_t now, uint64_t *n_removed) {
  if (!ft) return dpr_fail(DP_EINVAL, "null table");
  std::lock_guard<std::mutex> lk(ft->mu);
  if (int rc = pull_meta(ft)) return rc;
  Scratch &sc = ft->scr[0];
  unsigned long long cnt = 0;
  int rc = run(ft, "flow sweep", [&](hipStream_t st) {
    unsigned long long *dc = static_cast<unsigned long long *>(sc.get(2 * sizeof(cnt)));
    if (!dc) return dpr_fail(DP_ENOMEM, "flow scratch");
    if (hipMemsetAsync(dc, 0, 2 * sizeof(cnt), st) != hipSuccess) return dpr_fail(DP_EIO, "memset");
    const uint32_t b = blocks_for(ft->nslots) < 4096 ? blocks_for(ft->nslots) : 4096;
    hipLaunchKernelGGL(fl_sweep_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, now, dc);
    if (hipMemcpyAsync(&cnt, dc, sizeof(cnt), hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow sweep copy");
    // the tombstones the timers left, wherever they end a cluster
    hipLaunchKernelGGL(fl_reclaim_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, dc + 1);
    return 0;
  });
  if (rc) return rc;
  ft->len -= cnt;
  if (n_removed) *n_removed = cnt;
  return push_meta(ft);
}

int dp_flow_count(dp_flow_table_t *ft, uint64_t *len, uint64_t *active) {
  if (!ft) return dpr_fail(DP_EINVAL, "null table");
  std::lock_guard<std::mutex> lk(ft->mu);
  Scratch &sc = ft->scr[0];
  unsigned long long c[2] = {0, 0};
  int rc = run(ft, "flow count", [&](hipStream_t st) {
    unsigned long long *dc = static_cast<unsigned long long *>(sc.get(sizeof(c)));
    if (!dc) return dpr_fail(DP_ENOMEM, "flow scratch");
    if (hipMemsetAsync(dc, 0, sizeof(c), st) != hipSuccess) return dpr_fail(DP_EIO, "memset");
    const uint32_t b = blocks_for(ft->nslots) < 4096 ? blocks_for(ft->nslots) : 4096;
    hipLaunchKernelGGL(fl_count_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, dc);
    if (hipMemcpyAsync(c, dc, sizeof(c), hipMemcpyDeviceToHost, st) != hipSuccess)
      return dpr_fail(DP_EIO, "flow count copy");
    return 0;
  });
  if (rc) return rc;
  if (len) *len = c[0];
  if (active) *active = c[1];
  return 0;
}

}  // extern "C"

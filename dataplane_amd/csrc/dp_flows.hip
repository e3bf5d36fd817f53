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

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <map>
#include <unordered_set>
#include <string>
#include <vector>

#include "../../include/dpgpu.h"
#include "dp_flows_rt.h"
#include "dp_masq.h"

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
  if (s.flags & dpf::kFlagMasq) {  // MasqueradeState (nat/src/masquerade/state.rs:13-20)
    o.masq = (uint8_t)(s.pf & 0xffu);
    o.pf_status = (uint8_t)((s.pf >> 8) & 0xffu);
    o.pf_port = (uint16_t)(s.pf >> 16);
    o.pf_family = (uint8_t)s.pf_fam;
    for (int j = 0; j < 4; j++)
      for (int b = 0; b < 4; b++) o.pf_ip[4 * j + b] = (uint8_t)(s.pf_ip[j] >> (24 - 8 * b));
    if (s.pf_fam == 4) for (int b = 4; b < 16; b++) o.pf_ip[b] = 0;
    o.masq_alloc = s.mq_rec != 0;
    o.idle_timeout_s = s.pf_rule;
  }
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

// A flow leaving the table drops its FlowInfo, and with it the allocation its
// masquerade state owns (the Drop of its AllocatedPort, port_alloc.rs:
// 553-565): the (address record, port) goes on the call's release list, which
// the release kernels work through afterwards: the entries chained per address
// record and port block (fl_rel_link_k), each block's releases by one lane
// (fl_rel_run_k: a block's bitmap and count are its own, the address's
// counters atomic), then the addresses left
// without a block leave their region's list and bitmap one by one
// (fl_rel_kill_k: shared state; their order changes only which free record a
// later address takes).  false: the list is full -- the caller keeps the
// flow for a later round.
struct MqRel {
  uint32_t gen;   // the table's allocator generation (allocations of older ones are gone)
  uint32_t cap;
  uint32_t *cnt;  // [0] entries appended (may pass cap)
  uint32_t *list; // (record, port) pairs; nullptr: no allocator
};
__device__ __forceinline__ bool mq_depart(const MqRel &r, const FlowSlot &s) {
  if (!r.list || !(s.flags & dpf::kFlagMasq) || !s.mq_rec || s.mq_gen != r.gen) return true;
  const uint32_t k = atomicAdd(r.cnt, 1u);
  if (k >= r.cap) return false;
  r.list[2 * k] = s.mq_rec - 1;
  r.list[2 * k + 1] = s.pf >> 16;
  return true;
}
// per (address record, port block): the head of its chain of releases
// (kNone: none); per entry the next one; after the heads, the count of
// addresses to kill, then them
__global__ void __launch_bounds__(kTB) fl_rel_link_k(uint8_t *mq, const uint32_t *list, const uint32_t *cnt,
                                                    uint32_t cap, uint32_t *head, uint32_t *next) {
  const dpm::View V{mq};
  const uint32_t n = *cnt < cap ? *cnt : cap;
  for (uint32_t k = blockIdx.x * kTB + threadIdx.x; k < n; k += gridDim.x * kTB) {
    const uint32_t r = list[2 * k];
    next[k] = r < V.h().n_recs ? atomicExch(&head[256 * r + (list[2 * k + 1] >> 8)], k) : dpm::kNone;
  }
}
__global__ void __launch_bounds__(kTB) fl_rel_run_k(uint8_t *mq, const uint32_t *list, uint32_t *head,
                                                   const uint32_t *next, uint32_t *kill) {
  const dpm::View V{mq};
  const uint32_t nb = V.h().n_recs * 256;
  for (uint32_t b = blockIdx.x * kTB + threadIdx.x; b < nb; b += gridDim.x * kTB) {
    uint32_t k = head[b];
    if (k == dpm::kNone) continue;
    head[b] = dpm::kNone;  // (ready for the next call)
    bool dead = false;
    for (; k != dpm::kNone; k = next[k]) dead |= dpm::release_par(V, b >> 8, list[2 * k + 1]);
    if (dead) kill[1 + atomicAdd(&kill[0], 1u)] = b >> 8;
  }
}
// (without the chains' memory: every release by one lane, in list order)
__global__ void fl_release_k(uint8_t *mq, const uint32_t *list, const uint32_t *cnt, uint32_t cap) {
  const dpm::View V{mq};
  const uint32_t n = *cnt < cap ? *cnt : cap;
  for (uint32_t k = 0; k < n; k++) dpm::release(V, list[2 * k], list[2 * k + 1]);
}
__global__ void fl_rel_kill_k(uint8_t *mq, uint32_t *kill) {
  const dpm::View V{mq};
  for (uint32_t k = 0; k < kill[0]; k++) {
    const uint32_t r = kill[1 + k];
    if (V.recs()[r].region != dpm::kNone && V.recs()[r].live_blocks == 0) dpm::addr_kill(V, r);
  }
  kill[0] = 0;
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
                                                  uint64_t *refs, uint32_t *meta, MqRel rel) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  const InsRec r = recs[i];
  uint32_t sl = r.slot, old = 0;
  if (sl != dpf::kNoSlot) {
    old = slots[sl].state;
    (void)mq_depart(rel, slots[sl]);  // the replaced flow (one per record: room for all)
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
  s.mq_rec = 0;
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
                                                  const FKey *keys, uint32_t n, uint32_t *count, MqRel rel) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  uint32_t st;
  const uint32_t sl = probe(slots, mask, max_probe, keys[i], st);
  if (sl == dpf::kNoSlot) return;
  slots[sl].status = DP_FLOW_DETACHED;
  if (atomicCAS(&slots[sl].state, st, (st & ~3u) | dpf::FS_TOMB) != st) return;
  (void)mq_depart(rel, slots[sl]);  // one flow per key: room for all
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
// A flow whose allocation finds the release list full stays (Expired) for
// the next round of the same call.
__global__ void __launch_bounds__(kTB) fl_sweep_k(FlowSlot *slots, uint64_t nslots, uint64_t now,
                                                 unsigned long long *count, MqRel rel) {
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
    if (gone && mq_depart(rel, s) && atomicCAS(&s.state, st, (st & ~3u) | dpf::FS_TOMB) == st)
      atomicAdd(count, 1ull);
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

// A management call's release list for `cap` departures (counter zeroed on
// the stream); no list when the table has no allocator.  false: no memory.
bool rel_list(dp_flow_table *ft, uint32_t cap, hipStream_t st, MqRel &r) {
  r = MqRel{ft->mq_gen, cap, nullptr, nullptr};
  if (!ft->mq) return true;
  uint32_t *b = static_cast<uint32_t *>(ft->mq_rel.get(sizeof(uint32_t) * (2 * (size_t)(cap ? cap : 1) + 1)));
  if (!b || hipMemsetAsync(b, 0, sizeof(uint32_t), st) != hipSuccess) return false;
  r.cnt = b;
  r.list = b + 1;
  return true;
}
void rel_run(dp_flow_table *ft, const MqRel &r, hipStream_t st) {
  if (!r.list) return;
  // per-record chains: heads (all kNone between calls) and the kill list,
  // sized for the allocator's records; links per release entry
  const uint32_t nr = ft->mq_recs;
  uint32_t *h = static_cast<uint32_t *>(ft->mq_heads.get(sizeof(uint32_t) * (257 * (size_t)nr + 2)));
  uint32_t *nx = static_cast<uint32_t *>(ft->mq_next.get(sizeof(uint32_t) * ((size_t)r.cap + 1)));
  if (!h || !nx || !nr) {  // (no memory for the chains: one lane, in list order)
    hipLaunchKernelGGL(fl_release_k, dim3(1), dim3(1), 0, st, ft->mq, r.list, r.cnt, r.cap);
    return;
  }
  if (h != ft->mq_heads_at || nr != ft->mq_heads_n) {  // fresh buffer: no chain, no kill list
    (void)hipMemsetAsync(h, 0xff, sizeof(uint32_t) * 256 * (size_t)nr, st);
    (void)hipMemsetAsync(h + 256 * (size_t)nr, 0, sizeof(uint32_t) * (nr + 2), st);
    ft->mq_heads_at = h;
    ft->mq_heads_n = nr;
  }
  const uint32_t gb = blocks_for(r.cap) < 1024 ? blocks_for(r.cap) : 1024;
  hipLaunchKernelGGL(fl_rel_link_k, dim3(gb ? gb : 1), dim3(kTB), 0, st, ft->mq, r.list, r.cnt, r.cap, h, nx);
  const uint32_t rb = blocks_for(256ull * nr) < 4096 ? blocks_for(256ull * nr) : 4096;
  hipLaunchKernelGGL(fl_rel_run_k, dim3(rb ? rb : 1), dim3(kTB), 0, st, ft->mq, r.list, h, nx, h + 256 * (size_t)nr);
  hipLaunchKernelGGL(fl_rel_kill_k, dim3(1), dim3(1), 0, st, ft->mq, h + 256 * (size_t)nr);
}

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
      MqRel rel;
      if (!dr || !df || !rel_list(ft, (uint32_t)recs.size(), st, rel)) return dpr_fail(DP_ENOMEM, "flow scratch");
      hipLaunchKernelGGL(fl_insert_k, dim3(blocks_for(recs.size())), dim3(kTB), 0, st, ft->slots, ft->mask, dr,
                         (uint32_t)recs.size(), df, ft->d_meta, rel);
      rel_run(ft, rel, st);
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

// --------------------------------------------------------------------------
// masquerade allocator: build and sync (update_nat_allocator)
// --------------------------------------------------------------------------
typedef unsigned __int128 u128;

u128 pfx_first(const dp_prefix_t &p) {
  u128 v = 0;
  const int n = p.family == 4 ? 4 : 16;
  for (int i = 0; i < n; i++) v = (v << 8) | p.addr[i];
  return v;
}
u128 pfx_last(const dp_prefix_t &p) {
  const int w = p.family == 4 ? 32 : 128;
  const u128 host = p.len >= w ? (u128)0 : (p.len == 0 && w == 128 ? ~(u128)0 : (((u128)1 << (w - p.len)) - 1));
  return pfx_first(p) | host;
}
dpm::A128 to_a(u128 v) {
  dpm::A128 a;
  for (int i = 3; i >= 0; i--) { a.w[i] = (uint32_t)v; v >>= 32; }
  return a;
}

// decompose + regions_by_owner (apalloc/region.rs:43-130): the public space of
// one destination VPC's exposes cut into disjoint regions of constant owners
struct RegionSpec {
  u128 lo, hi;
  std::vector<size_t> owners;
};
std::vector<RegionSpec> decompose(const std::vector<std::vector<std::pair<u128, u128>>> &own) {
  std::vector<u128> c;
  for (auto &rs : own)
    for (auto &r : rs) {
      c.push_back(r.first);
      if (r.second != ~(u128)0) c.push_back(r.second + 1);
    }
  std::sort(c.begin(), c.end());
  c.erase(std::unique(c.begin(), c.end()), c.end());
  std::vector<RegionSpec> out;
  for (size_t i = 0; i < c.size(); i++) {
    const u128 s = c[i], e = i + 1 < c.size() ? c[i + 1] - 1 : ~(u128)0;
    std::vector<size_t> owners;
    for (size_t o = 0; o < own.size(); o++)
      for (auto &r : own[o]) if (r.first <= s && s <= r.second) { owners.push_back(o); break; }
    if (owners.empty()) continue;
    if (!out.empty() && out.back().hi + 1 == s && out.back().owners == owners) out.back().hi = e;
    else out.push_back(RegionSpec{s, e, owners});
  }
  return out;
}

// NatAllocator::new -> build_pools_generic (apalloc/setup.rs:158-204) into the
// dp_masq.h layout: per family, per destination VPC, per protocol the regions
// of its exposes' public prefixes (each its own NatPool), per expose a PoolSet
// of its regions (fewest sharers, widest, lowest first), per private prefix a
// PoolTable entry.  `used`: bytes through the address records (the records
// area is not initialised; a new address writes its whole record).
constexpr uint32_t kNeverUsed = dpm::kNone - 1;
std::vector<uint8_t> masq_build(const dpd::MasqConfig &cfg, int64_t genid, uint32_t gen) {
  struct EKey {
    uint32_t proto, src, dst;
    u128 lo, hi;
    bool operator<(const EKey &o) const {
      if (proto != o.proto) return proto < o.proto;
      if (src != o.src) return src < o.src;
      if (dst != o.dst) return dst < o.dst;
      if (lo != o.lo) return lo < o.lo;
      return hi < o.hi;
    }
  };
  std::map<EKey, uint32_t> table;  // add_pool_entries: a later expose's entry replaces
  std::vector<dpm::Set> sets;
  std::vector<uint32_t> setreg;
  std::vector<dpm::Region> regions;
  std::vector<dpm::Claim> claims;
  uint32_t bit_words = 0;
  uint64_t sum_cap = 0;
  for (int fam : {4, 6}) {
    std::map<uint32_t, std::vector<const dpd::MasqExpose *>> groups;  // by destination VPC
    for (auto &e : cfg.exposes) if (e.fam == fam) groups[e.dst_vni].push_back(&e);
    for (auto &g : groups) {
      for (uint32_t proto : {6u, 17u, fam == 4 ? 1u : 58u}) {
        std::vector<std::vector<std::pair<u128, u128>>> own;
        for (auto *e : g.second) {
          std::vector<std::pair<u128, u128>> rs;
          for (auto &p : e->pub) rs.push_back({pfx_first(p), pfx_last(p)});
          own.push_back(rs);
        }
        const auto specs = decompose(own);
        const uint32_t r0 = (uint32_t)regions.size();
        for (auto &R : specs) {
          dpm::Region x{};
          x.fam = (uint32_t)fam;
          const u128 span = R.hi - R.lo;
          x.cap = span >= DP_MASQ_REGION_ADDRS - 1 ? DP_MASQ_REGION_ADDRS : (uint32_t)span + 1;
          x.excl_wk = proto == 6 || proto == 17;
          x.start = to_a(R.lo);
          x.last = to_a(R.hi);
          x.claim_first = (uint32_t)claims.size();
          const uint32_t bit = proto == 6 ? DP_MASQ_TCP : proto == 17 ? DP_MASQ_UDP : 0u;
          for (size_t o : R.owners)
            for (auto &c : g.second[o]->claims)
              if (c.protos & bit) {
                dpm::Claim k{};
                k.net = to_a(pfx_first(c.prefix));
                k.fam = c.prefix.family;
                k.len = c.prefix.len;
                k.lo = c.lo;
                k.hi = c.hi;
                claims.push_back(k);
              }
          x.claim_n = (uint32_t)claims.size() - x.claim_first;
          x.head = x.tail = dpm::kNone;
          x.bits = bit_words;
          x.hint = 0;
          bit_words += (x.cap + 31) / 32;
          sum_cap += x.cap;
          regions.push_back(x);
        }
        for (size_t o = 0; o < g.second.size(); o++) {
          std::vector<size_t> mine;
          for (size_t r = 0; r < specs.size(); r++)
            if (std::find(specs[r].owners.begin(), specs[r].owners.end(), o) != specs[r].owners.end())
              mine.push_back(r);
          std::stable_sort(mine.begin(), mine.end(), [&](size_t a, size_t b) {
            const auto &x = specs[a], &y = specs[b];
            if (x.owners.size() != y.owners.size()) return x.owners.size() < y.owners.size();
            const u128 lx = x.hi - x.lo, ly = y.hi - y.lo;
            if (lx != ly) return lx > ly;
            return x.lo < y.lo;
          });
          dpm::Set S{};
          S.idle_ns = g.second[o]->idle_ns;
          S.first_reg = (uint32_t)setreg.size();
          S.n_reg = (uint32_t)mine.size();
          for (size_t r : mine) setreg.push_back(r0 + (uint32_t)r);
          const uint32_t si = (uint32_t)sets.size();
          sets.push_back(S);
          for (auto &p : g.second[o]->priv)
            table[EKey{proto | ((uint32_t)fam << 8), g.second[o]->src_vni, g.first, pfx_first(p), pfx_last(p)}] = si;
        }
      }
    }
  }
  // the table's runs: one per (protocol | family, source, destination)
  std::vector<dpm::Ent> ents;
  std::vector<dpm::KeySlot> runs;
  for (auto &kv : table) {
    const EKey &k = kv.first;
    if (runs.empty() || runs.back().proto != k.proto || runs.back().src != k.src ||
        (runs.back().dst & 0x7fffffffu) != k.dst)
      runs.push_back(dpm::KeySlot{k.proto, k.src, k.dst | 0x80000000u, (uint32_t)ents.size(), 0, {0, 0, 0}});
    runs.back().n++;
    dpm::Ent e{};
    e.lo = to_a(k.lo);
    e.hi = to_a(k.hi);
    e.set = kv.second;
    ents.push_back(e);
  }
  uint32_t ksz = 1;
  while (ksz < 2 * runs.size() + 2) ksz <<= 1;
  std::vector<dpm::KeySlot> keys(ksz);
  for (auto &r : runs) {
    uint32_t i = dpm::kmix(r.proto, r.src, r.dst & 0x7fffffffu) & (ksz - 1);
    while (keys[i].dst >> 31) i = (i + 1) & (ksz - 1);
    keys[i] = r;
  }
  const uint32_t n_recs = (uint32_t)std::min<uint64_t>(sum_cap, DP_MASQ_ADDRS);
  dpm::Header H{};
  H.magic = dpm::kMagic;
  H.gen = gen;
  H.genid = genid;
  H.key_mask = ksz - 1;
  H.n_keys = (uint32_t)runs.size();
  H.n_regions = (uint32_t)regions.size();
  H.n_recs = n_recs;
  H.free_top = n_recs;
  H.live = 0;
  H.max_live = DP_MASQ_ADDRS;
  H.randomize = cfg.randomize ? 1u : 0u;
  H.seed = cfg.seed;
  uint64_t off = (sizeof(dpm::Header) + 63) & ~63ull;
  auto place = [&](uint64_t bytes) { const uint64_t o = off; off = (off + bytes + 63) & ~63ull; return o; };
  H.o_keys = place(sizeof(dpm::KeySlot) * keys.size());
  H.o_ents = place(sizeof(dpm::Ent) * ents.size());
  H.o_sets = place(sizeof(dpm::Set) * sets.size());
  H.o_setreg = place(sizeof(uint32_t) * setreg.size());
  H.o_regions = place(sizeof(dpm::Region) * regions.size());
  H.o_claims = place(sizeof(dpm::Claim) * claims.size());
  H.o_bits = place(sizeof(uint32_t) * bit_words);
  H.o_free = place(sizeof(uint32_t) * n_recs);
  H.o_recs = place(0);
  H.bytes = H.o_recs + sizeof(dpm::Addr) * (uint64_t)n_recs;
  std::vector<uint8_t> b(H.bytes, 0);
  memcpy(b.data(), &H, sizeof H);
  // records never handed out are marked so (the upload stops after the last one used)
  dpm::Addr *ra = reinterpret_cast<dpm::Addr *>(b.data() + H.o_recs);
  for (uint32_t i = 0; i < n_recs; i++) ra[i].region = kNeverUsed;
  auto copy = [&](uint64_t o, const void *p, size_t n) { if (n) memcpy(b.data() + o, p, n); };
  copy(H.o_keys, keys.data(), sizeof(dpm::KeySlot) * keys.size());
  copy(H.o_ents, ents.data(), sizeof(dpm::Ent) * ents.size());
  copy(H.o_sets, sets.data(), sizeof(dpm::Set) * sets.size());
  copy(H.o_setreg, setreg.data(), sizeof(uint32_t) * setreg.size());
  copy(H.o_regions, regions.data(), sizeof(dpm::Region) * regions.size());
  copy(H.o_claims, claims.data(), sizeof(dpm::Claim) * claims.size());
  uint32_t *bw = reinterpret_cast<uint32_t *>(b.data() + H.o_bits);
  for (auto &R : regions)
    for (uint32_t o = 0; o < R.cap; o++) bw[R.bits + (o >> 5)] |= 1u << (o & 31);
  // the free records, popped lowest first
  uint32_t *fs = reinterpret_cast<uint32_t *>(b.data() + H.o_free);
  for (uint32_t i = 0; i < n_recs; i++) fs[i] = n_recs - 1 - i;
  return b;
}

// A masquerading flow holding an allocation, as check_masquerading_flow sees it
struct MqFlow {
  uint32_t slot, state, vni, fk;
  uint32_t src[4];   // key source (address bytes as stored)
  uint32_t dst_vni, pf, fam, flags;
  uint32_t ip[4];    // use_ip (big-endian words)
};
struct MqDecision {
  uint32_t slot, state, rec;  // rec: the new allocation's record, kNone: invalidate the pair
};

// Active masquerading flows with an allocation and another generation than the
// new allocator's (the flows check_masquerading_flow re-reserves).
__global__ void __launch_bounds__(kTB) mq_collect_k(const FlowSlot *slots, uint64_t nslots, int64_t genid,
                                                   MqFlow *out, uint32_t cap, uint32_t *cnt) {
  for (uint64_t i = blockIdx.x * (uint64_t)kTB + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * kTB) {
    const FlowSlot &s = slots[i];
    const uint32_t st = s.state;
    if ((st & 3u) != dpf::FS_FULL || s.status != DP_FLOW_ACTIVE || !(s.flags & dpf::kFlagMasq) || !s.mq_rec ||
        s.genid == genid)
      continue;
    const uint32_t k = atomicAdd(cnt, 1u);
    if (k >= cap) continue;
    MqFlow f;
    f.slot = (uint32_t)i;
    f.state = st;
    f.vni = s.src_vni;
    f.fk = s.fk;
    for (int j = 0; j < 4; j++) { f.src[j] = s.src[j]; f.ip[j] = s.pf_ip[j]; }
    f.dst_vni = s.dst_vni;
    f.pf = s.pf;
    f.fam = s.pf_fam;
    f.flags = s.flags;
    out[k] = f;
  }
}
// set_genid_pair / invalidate_pair of the re-reserved / dropped flows
__global__ void __launch_bounds__(kTB) mq_apply_k(FlowSlot *slots, uint32_t mask, const MqDecision *d, uint32_t n,
                                                 int64_t genid, uint32_t gen) {
  const uint32_t i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  const MqDecision x = d[i];
  FlowSlot &s = slots[x.slot];
  if (s.state != x.state) return;
  const bool rel = s.related <= mask && slots[s.related].state == s.related_tag;
  if (x.rec == dpm::kNone) {
    s.status = DP_FLOW_CANCELLED;
    if (rel) slots[s.related].status = DP_FLOW_CANCELLED;
  } else {
    s.mq_rec = x.rec + 1;
    s.mq_gen = gen;
    s.genid = genid;
    if (rel) slots[s.related].genid = genid;
  }
}
// upgrade_all_masquerading_flows (flows.rs:30-44)
__global__ void __launch_bounds__(kTB) mq_upgrade_k(FlowSlot *slots, uint64_t nslots, int64_t genid) {
  for (uint64_t i = blockIdx.x * (uint64_t)kTB + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * kTB) {
    FlowSlot &s = slots[i];
    if ((s.state & 3u) == dpf::FS_FULL && s.status == DP_FLOW_ACTIVE && (s.flags & dpf::kFlagMasq)) s.genid = genid;
  }
}
// invalidate_masquerade_flows (flows.rs:19-27): every masquerading flow's pair
__global__ void __launch_bounds__(kTB) mq_drop_k(FlowSlot *slots, uint64_t nslots, uint32_t mask) {
  for (uint64_t i = blockIdx.x * (uint64_t)kTB + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * kTB) {
    FlowSlot &s = slots[i];
    if ((s.state & 3u) != dpf::FS_FULL || !(s.flags & dpf::kFlagMasq)) continue;
    s.status = DP_FLOW_CANCELLED;
    if (s.related <= mask && slots[s.related].state == s.related_tag) slots[s.related].status = DP_FLOW_CANCELLED;
  }
}

bool covers(const dp_prefix_t &p, int fam, u128 a) { return p.family == fam && pfx_first(p) <= a && a <= pfx_last(p); }

}  // namespace

int dpf_masq_sync(dp_flow_table *ft, const std::shared_ptr<const dpd::MasqConfig> &cfg, int64_t genid,
                  uint64_t serial) {
  if (!cfg || ft->mq_serial == serial) return 0;
  const uint32_t b = blocks_for(ft->nslots) < 4096 ? blocks_for(ft->nslots) : 4096;
  if (ft->mq && ft->mq_cfg && ft->mq_cfg->same(*cfg)) {
    // the same config: the allocator stays, its flows move to the new generation
    int rc = run(ft, "masquerade upgrade", [&](hipStream_t st) {
      if (hipMemcpyAsync(ft->mq + offsetof(dpm::Header, genid), &genid, sizeof genid, hipMemcpyHostToDevice, st) !=
          hipSuccess)
        return dpr_fail(DP_EIO, "allocator genid");
      hipLaunchKernelGGL(mq_upgrade_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, genid);
      return 0;
    });
    if (!rc) ft->mq_serial = serial;
    return rc;
  }
  if (cfg->exposes.empty()) {
    if (ft->mq) {
      int rc = run(ft, "masquerade drop", [&](hipStream_t st) {
        hipLaunchKernelGGL(mq_drop_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, ft->mask);
        return 0;
      });
      if (rc) return rc;
      (void)hipFree(ft->mq);
      ft->mq = nullptr;
      ft->mq_recs = 0;
      ft->mq_cfg.reset();
      ft->mq_gen = 0;
    }
    ft->mq_serial = serial;
    return 0;
  }
  const uint32_t gen = ft->mq_next_gen++;
  std::vector<uint8_t> buf = masq_build(*cfg, genid, gen);
  // (the device copy is the whole layout; records past the ones handed out are
  // written by the first allocation that takes them)
  const dpm::View V{buf.data()};
  // the flows to carry over
  Scratch &sa = ft->scr[0], &sb = ft->scr[1];
  uint32_t n = 0;
  std::vector<MqFlow> flows;
  for (int pass = 0; pass < 2; pass++) {
    const uint32_t cap = pass ? n : 0;
    flows.resize(cap);
    uint32_t got = 0;
    int rc = run(ft, "masquerade flows", [&](hipStream_t st) {
      uint32_t *dc = static_cast<uint32_t *>(sa.get(sizeof(uint32_t)));
      MqFlow *df = static_cast<MqFlow *>(sb.get(sizeof(MqFlow) * (cap ? cap : 1)));
      if (!dc || !df) return dpr_fail(DP_ENOMEM, "flow scratch");
      if (hipMemsetAsync(dc, 0, sizeof(uint32_t), st) != hipSuccess) return dpr_fail(DP_EIO, "memset");
      hipLaunchKernelGGL(mq_collect_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, genid, df, cap, dc);
      if (hipMemcpyAsync(&got, dc, sizeof got, hipMemcpyDeviceToHost, st) != hipSuccess ||
          (cap && hipMemcpyAsync(flows.data(), df, sizeof(MqFlow) * cap, hipMemcpyDeviceToHost, st) != hipSuccess))
        return dpr_fail(DP_EIO, "masquerade flows copy");
      return 0;
    });
    if (rc) return rc;
    n = got;
    if (!n) break;
  }
  // check_masquerading_flow for each, in ascending (address, port) order
  auto ip_bytes = [](const MqFlow &f, uint8_t out[16]) {
    memset(out, 0, 16);
    for (int j = 0; j < (f.fam == 4 ? 1 : 4); j++)
      for (int k = 0; k < 4; k++) out[4 * j + k] = (uint8_t)(f.ip[j] >> (24 - 8 * k));
  };
  std::stable_sort(flows.begin(), flows.end(), [&](const MqFlow &x, const MqFlow &y) {
    uint8_t a[16], c[16];
    ip_bytes(x, a);
    ip_bytes(y, c);
    const int r = memcmp(a, c, 16);
    if (r) return r < 0;
    return (x.pf >> 16) < (y.pf >> 16);
  });
  std::vector<MqDecision> dec;
  for (const MqFlow &f : flows) {
    const int kfam = (int)(f.fk & 0xffu), kind = (int)(f.fk >> 8);
    u128 ip = 0, src = 0;
    for (int j = 0; j < (f.fam == 4 ? 1 : 4); j++) ip = (ip << 32) | f.ip[j];
    uint8_t sb8[16];
    memcpy(sb8, f.src, 16);
    for (int j = 0; j < (kfam == 4 ? 4 : 16); j++) src = (src << 8) | sb8[j];
    bool peering = false, ip_ok = false, compatible = false;
    for (auto &e : cfg->exposes) {
      if (e.src_vni != f.vni || e.dst_vni != f.dst_vni) continue;
      peering = true;
      bool pub = false;
      for (auto &q : e.pub) pub |= covers(q, (int)f.fam, ip);
      if (!pub) continue;
      ip_ok = true;
      bool pri = false;
      for (auto &q : e.priv) pri |= covers(q, kfam, src);
      if (pri) { compatible = true; break; }
    }
    uint32_t rec = dpm::kNone;
    if (peering && ip_ok && compatible) {
      const uint32_t proto = kind == DP_FLOW_TCP ? 6u : kind == DP_FLOW_UDP ? 17u : kfam == 4 ? 1u : 58u;
      const uint32_t set = dpm::lookup(V, proto | ((uint32_t)kfam << 8), f.vni, f.dst_vni, to_a(src));
      uint32_t r = 0;
      if (set != dpm::kNone &&
          dpm::set_reserve(V, set, to_a(ip), f.pf >> 16, (f.flags & dpf::kFlagMasqIdent) != 0, r) == dpm::OK)
        rec = r;
    }
    dec.push_back(MqDecision{f.slot, f.state, rec});
  }
  uint8_t *dev = nullptr;
  if (hipSetDevice(ft->device) != hipSuccess || hipMalloc(&dev, buf.size()) != hipSuccess)
    return dpr_fail(DP_ENOMEM, "masquerade allocator");
  int rc = run(ft, "masquerade allocator", [&](hipStream_t st) {
    // the records handed out sit lowest (the free stack pops them in order)
    uint32_t hi = 0;
    while (hi < V.h().n_recs && V.recs()[hi].region != kNeverUsed) hi++;
    const uint64_t used = V.h().o_recs + sizeof(dpm::Addr) * (uint64_t)hi;
    if (hipMemcpyAsync(dev, buf.data(), used, hipMemcpyHostToDevice, st) != hipSuccess)
      return dpr_fail(DP_EIO, "masquerade allocator upload");
    if (!dec.empty()) {
      MqDecision *dd = upload(sa, dec.data(), dec.size(), st);
      if (!dd) return dpr_fail(DP_ENOMEM, "flow scratch");
      hipLaunchKernelGGL(mq_apply_k, dim3(blocks_for(dec.size())), dim3(kTB), 0, st, ft->slots, ft->mask, dd,
                         (uint32_t)dec.size(), genid, gen);
    }
    return 0;
  });
  if (rc) { (void)hipFree(dev); return rc; }
  if (ft->mq) (void)hipFree(ft->mq);
  ft->mq = dev;
  ft->mq_gen = gen;
  ft->mq_recs = reinterpret_cast<const dpm::Header *>(buf.data())->n_recs;
  ft->mq_cfg = cfg;
  ft->mq_serial = serial;
  return 0;
}

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
  dpr_forget_flow_table(ft);
  (void)hipSetDevice(ft->device);
  if (ft->burst_armed) (void)hipEventSynchronize(ft->last_burst);
  (void)hipStreamSynchronize(ft->stream);
  (void)hipFree(ft->slots);
  (void)hipFree(ft->d_meta);
  if (ft->mq) (void)hipFree(ft->mq);
  ft->mq_rel.release();
  ft->mq_heads.release();
  ft->mq_next.release();
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
    MqRel rel;
    if (!dk || !dc || !rel_list(ft, n, st, rel)) return dpr_fail(DP_ENOMEM, "flow scratch");
    if (hipMemsetAsync(dc, 0, sizeof(uint32_t), st) != hipSuccess) return dpr_fail(DP_EIO, "memset");
    if (n) {
      hipLaunchKernelGGL(fl_remove_k, dim3(blocks_for(n)), dim3(kTB), 0, st, ft->slots, ft->mask, ft->max_probe,
                         dk, n, dc, rel);
      rel_run(ft, rel, st);
    }
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
  // rounds of at most kRelCap allocations released (a flow that found the
  // list full is Expired and goes in a later round)
  constexpr uint32_t kRelCap = 1u << 20;
  const uint32_t cap = ft->nslots < kRelCap ? (uint32_t)ft->nslots : kRelCap;
  uint32_t appended = 0;
  int rc = 0;
  do {
    rc = run(ft, "flow sweep", [&](hipStream_t st) {
      unsigned long long *dc = static_cast<unsigned long long *>(sc.get(2 * sizeof(cnt)));
      MqRel rel;
      if (!dc || !rel_list(ft, cap, st, rel)) return dpr_fail(DP_ENOMEM, "flow scratch");
      if (hipMemsetAsync(dc, 0, 2 * sizeof(cnt), st) != hipSuccess) return dpr_fail(DP_EIO, "memset");
      const uint32_t b = blocks_for(ft->nslots) < 4096 ? blocks_for(ft->nslots) : 4096;
      hipLaunchKernelGGL(fl_sweep_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, now, dc, rel);
      rel_run(ft, rel, st);
      unsigned long long c = 0;
      appended = 0;
      if (hipMemcpyAsync(&c, dc, sizeof(c), hipMemcpyDeviceToHost, st) != hipSuccess ||
          (rel.cnt && hipMemcpyAsync(&appended, rel.cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess))
        return dpr_fail(DP_EIO, "flow sweep copy");
      if (hipStreamSynchronize(st) != hipSuccess) return dpr_fail(DP_EIO, "flow sweep");
      cnt += c;
      // the tombstones the timers left, wherever they end a cluster
      hipLaunchKernelGGL(fl_reclaim_k, dim3(b), dim3(kTB), 0, st, ft->slots, ft->nslots, dc + 1);
      return 0;
    });
  } while (!rc && appended > cap);
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

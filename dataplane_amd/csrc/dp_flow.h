// SPDX-License-Identifier: Apache-2.0
//
// Device flow table (include/dpgpu.h "Flow table"): the reference's
// FlowTable (flow-entry/src/flow_table/table.rs:24-330) as one open-addressing
// array of 128-byte slots in HBM -- one slot is one L2 line, so a probe is one
// memory transaction and the key (first 48 bytes) arrives with the state word.
// Shared by the management kernels (dp_flows.hip) and the pipeline kernel's
// flow-aware stages (dp_kernel.hip).
#pragma once
#include <stdint.h>

namespace dpf {

// slot state (low 2 bits of FlowSlot::state); the upper 30 bits are a fill tag
// that changes on every fill, so a (slot, tag) ref names one stored FlowInfo
enum : uint32_t { FS_EMPTY = 0, FS_BUSY = 1, FS_FULL = 2, FS_TOMB = 3 };
constexpr uint32_t kNoSlot = 0xffffffffu;
constexpr uint32_t kIdleMark = 0xffffffffu;

struct alignas(128) FlowSlot {
  uint32_t state;       // FS_* | tag << 2
  uint32_t src_vni;     // key: FlowKey.src_vpcd (0 = None)
  uint32_t fk;          // key: family | kind << 8
  uint32_t ports;       // key: sport << 16 | dport
  uint32_t src[4];      // key: address bytes as given (v4: first word, rest 0)
  uint32_t dst[4];
  uint32_t status;      // FlowStatus
  uint32_t flags;       // FlowInfoFlags
  uint32_t dst_vni;     // FlowInfoLocked.dst_vpcd
  uint32_t related;     // slot of the related flow (kNoSlot: none)
  uint32_t related_tag; // that slot's state word when the pair was made
  uint32_t mark;        // burst-local invalidation mark (kIdleMark between bursts)
  int64_t genid;
  uint64_t expires_at;
  uint32_t pad[10];
};
static_assert(sizeof(FlowSlot) == 128, "one L2 line per slot");

// the 11 key words of a FlowKey, in slot order
struct FKey {
  uint32_t w[11];
};

__host__ __device__ inline uint32_t fkey_hash(const FKey &k) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
#pragma unroll
  for (int i = 0; i < 11; i++) {
    h = (h ^ k.w[i]) * 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  h *= 0xc4ceb9fe1a85ec53ull;
  return (uint32_t)(h ^ (h >> 29));
}

// The launch-time view of a flow table for one burst.
struct FlowCtx {
  FlowSlot *slots;
  uint32_t mask;        // slots - 1
  uint32_t n;           // packets of the burst
  uint32_t max_probe;   // probe bound (dp_flow_table::max_probe)
  uint32_t pad;
  // invalidation events: [0] count, then (slot, state word) of each
  // invalidated flow (<= 2 per packet); the state word is the fill the event
  // is about, so an event never touches a later fill of the slot
  uint32_t *events;
  // ACL decisions that rest on a flow's validity (acl = 6): [0] count, then
  // SensRec records
  uint32_t *sens;
  int64_t genid;        // the burst's PipelineData genid
};

// A packet whose ACL verdict was "allow: reply of a flow-scope-allowed flow";
// if its flow turns out invalidated earlier in the burst, the verdict is the
// peering default instead (dp_flow_fixup), with the meta as it was at the ACL.
struct SensRec {
  uint32_t idx;         // packet index
  uint32_t slot;        // its flow
  uint32_t meta_flags;  // at the ACL
  uint32_t oif;         // at the ACL (0: None)
  uint32_t fib_entry;   // at the ACL
  uint32_t def_acl;     // the default verdict: out.acl code 3 / 4 / 5
  uint32_t related;     // the flow's related slot and its state when paired
  uint32_t related_tag;
  uint32_t dst_vni;     // PacketMeta at the ACL: dst_vpcd, vrf (bit 31: Some), the nh_addr source
  uint32_t vrf;
  uint32_t nh_ref;
  uint32_t pad;
};

__host__ __device__ inline uint64_t make_ref(uint32_t slot, uint32_t state) {
  return ((uint64_t)(state >> 2) << 32) | slot;
}

}  // namespace dpf

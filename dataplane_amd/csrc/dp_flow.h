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
// FlowSlot::flags bits (above the FlowInfoFlags of dpgpu.h): the flow holds
// port-forwarding state (FlowInfoLocked.port_fw_state is Some), masquerade
// state (nat/src/masquerade/state.rs:13-20), whose use_port is an ICMP
// identifier (NatPort::Identifier)
constexpr uint32_t kFlagPf = 1u << 8;
constexpr uint32_t kFlagMasq = 1u << 9;
constexpr uint32_t kFlagMasqIdent = 1u << 10;

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
  // PortFwState (nat/src/portfw/flow_state.rs:29-35), valid with kFlagPf:
  // action (dp_pf_action) | NatFlowStatus << 8 | use_port << 16, the entry id
  // its Weak names, use_ip (big-endian words; v4 in word 0).  MasqueradeState
  // (kFlagMasq) in the same words: action | status << 8 | use_port << 16,
  // the idle timeout in seconds, use_ip
  uint32_t pf;
  uint32_t pf_rule;
  uint32_t pf_ip[4];
  uint32_t pf_fam;
  // the allocation a masquerading SrcNat flow owns (its AllocatedPort):
  // address record + 1 (0: none) and the allocator generation it lives in
  uint32_t mq_rec;
  uint32_t mq_gen;
  // the burst (FlowCtx::burst) in which a masquerading record of this flow's
  // pair may change its NatFlowStatus (dp_nat_mark: its refreshes are then
  // not order-free)
  uint32_t nat_tag;
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

// One packet that reached PortForwarder (nat/src/portfw/nf.rs:373-397) in
// the burst's first pass: what the sequential port-forwarding pass
// (dp_nat_prep, dp_nat_resolve) needs, then its decision for the replay pass.
struct PfReq {
  uint32_t idx;          // packet index
  uint32_t bits;         // kPq* below
  uint32_t slot, state;  // the flow FlowLookup attached (kNoSlot: none) and its fill
  uint32_t status0;      // its FlowStatus and flags as the burst started
  uint32_t fflags0;
  uint32_t src_vni;      // PacketMeta.src_vpcd (0: None)
  uint32_t proto;        // IP next header | family << 8 | TCP flags << 16
  uint32_t ports;        // sport << 16 | dport (TCP / UDP)
  uint32_t src[4], dst[4];  // current addresses (big-endian words)
  uint32_t ikey[11];     // PacketMeta.flow_key (kPqIkey): the key before static NAT
  uint32_t acl_def;      // ACL: the peering default verdict of a kPqSens packet (out.acl 3/4/5)
  uint32_t acl_rule6;    // ... and the rule of its verdict 6
  uint32_t dst_vni0, related0, related_tag0;  // the attached flow as the burst started
  int64_t genid0;
  uint32_t dst_vni;      // PacketMeta.dst_vpcd at the NAT stages
  // decision (dp_nat_resolve -> replay)
  uint32_t verdict;      // PortForwarder: DoneReason to drop with, or kPfForward
  uint32_t nat;          // dp_pf_action | port << 16
  uint32_t nat_ip[4];
  uint32_t acl_over;     // 0, or the ACL verdict the sens check left (out.acl code)
  uint32_t mverdict;     // Masquerade: DoneReason, or kPfForward
  uint32_t mnat;         // dp_pf_action | ident (1 << 8) | port << 16
  uint32_t mnat_ip[4];
  // the first pass's ACL outcome (out.acl code, rule): the replay takes it
  // (and the flow filter's, dst_vni and the kPq requirement bits) instead of
  // classifying again
  uint32_t acl_code;
  uint32_t acl_rule;
};
constexpr uint32_t kPqReached = 1u << 0;  // the packet reached PortForwarder (else dropped on the way)
constexpr uint32_t kPqTcp = 1u << 1;
constexpr uint32_t kPqUdp = 1u << 2;
constexpr uint32_t kPqIkey = 1u << 3;
constexpr uint32_t kPqSens = 1u << 4;     // ACL verdict 6 (reply of a flow-scope-allowed flow)
constexpr uint32_t kPqRelated = 1u << 5;  // related / related_tag valid at attach
constexpr uint32_t kPqEth = 1u << 6;
constexpr uint32_t kPqSnatSrc = 1u << 7;  // PacketMeta requires static NAT of the source / destination
constexpr uint32_t kPqSnatDst = 1u << 8;
constexpr uint32_t kPqPf = 1u << 9;       // PortForwarder runs on it (REQ_PORT_FORWARDING)
constexpr uint32_t kPqMasq = 1u << 10;    // Masquerade runs on it (REQ_MASQUERADE)
constexpr uint32_t kPqIcmp = 1u << 11;    // an ICMP v4 / v6 header
constexpr uint32_t kPqQuery = 1u << 12;   // its flow key is an ICMP query's (echo, code 0)
// the masquerading burst's split pass (dp_nat_resolve / dp_nat_lane): the
// record runs on the burst's one allocating lane; PortForwarder's part of it
// already ran (its connection's lane left it there)
constexpr uint32_t kPqLane = 1u << 13;
constexpr uint32_t kPqPfDone = 1u << 14;
// a steady refresh dp_nat_prep resolved in place (its replay may start then)
constexpr uint32_t kPqSteady = 1u << 15;
constexpr uint32_t kPfForward = 0xffu;

// words of FlowCtx::pf_cnt
constexpr uint32_t kCntWords = 40;
#define DPF_CNT_WORDS 40

// The launch-time view of a flow table for one burst.
struct FlowCtx {
  FlowSlot *slots;
  uint32_t mask;        // slots - 1
  uint32_t n;           // packets of the burst
  uint32_t max_probe;   // unused (the bound lives in tmeta[0])
  uint32_t pad;
  // invalidation events: [0] count, then (slot, state word) of each
  // invalidated flow (<= 2 per packet); the state word is the fill the event
  // is about, so an event never touches a later fill of the slot
  uint32_t *events;
  // ACL decisions that rest on a flow's validity (acl = 6): [0] count, then
  // SensRec records
  uint32_t *sens;
  int64_t genid;        // the burst's PipelineData genid
  // device words of the table: [0] probe bound (largest displacement of any
  // stored flow), [2..3] FlowTable::len (u64)
  uint32_t *tmeta;
  uint64_t capacity;    // FlowTable capacity
  uint64_t hard;        // slots - slots / 8: no new slot beyond it
  uint64_t now;         // the flow clock (DP_OPT_CLOCK)
  // port forwarding: records, [0] count then packet -> record index, the
  // bitmap of packets that reached PortForwarder (+ its summary, 1 bit per
  // 1024 packets), the order of the records (resolve), replaced fills
  PfReq *pf;
  uint32_t *pf_cnt;     // [0] records, [1] replay packets, [2] replaced fills, [3] releases, [4..15] below
  uint32_t *pf_of;      // packet -> record
  uint32_t *pf_bits;
  uint32_t *pf_sum;
  uint32_t *pf_order;
  uint32_t *pf_repl;    // (slot, old state, packet index, old mark) of each fill replaced
  uint32_t replay;      // the replay pass: 1 packets pf_order[0..pf_cnt[1]), 4 the steady refreshes
                        // among them (kPqSteady), 2 the others off a masquerade split's allocating
                        // lane, 3 the lane's (lane_order[0..pf_cnt[11]))
  // masquerade: the table's allocator (dp_masq.h; nullptr: none) and its
  // generation, the allocations of fills replaced in the burst (record,
  // port), released when the sequential pass ends
  uint8_t *mq;
  uint32_t mq_gen;
  uint32_t *mq_rel;
  // the NAT pass's connections (dp_nat_prep / dp_nat_resolve): per hash slot
  // (burst << 32 | connection key) and (burst << 32 | its last record), per
  // record (packet index << 32 | the connection's record before it), the
  // slots claimed this burst; [4] their count, [5] a record the parallel
  // pass cannot take, [6..7] the table length as the pass starts.
  // Masquerade (dp_nat_resolve, dp_nat_lane): [8] masquerade records, [9]
  // PortForwarder records, [10] a masqueraded packet whose peer could
  // masquerade back (pfw::masq_back), [11] records on the allocating lane,
  // [12] the mode that ran (1 one lane, 2 connections, 3 split, 4 connections
  // near the capacity, 5 connections beside the split), [13] records
  // a connection lane left to the allocating lane, [14] allocations served in
  // wave batches, [15] allocations on the lane alone, [16] pairs the split
  // pass could not create (never: it runs only with room; counters for tests).
  // Port forwarding without room for every pair (dp_nat_admit_*): [17] a
  // connection whose creations the admission pass cannot foresee.  [18]
  // records the allocating lane ran alone (live flow state, or no room);
  // [19..22] its time in plans, allocations, pairs and records alone (1024
  // clock64 ticks), [23..25] the allocations' parts (the set's address and
  // block, serving the records, the block's update), [26] allocation steps,
  // [27] a steady refresh in the burst (dp_nat_prep), [28] an initial key of
  // the lane's allocating records repeats, [29] a lane record runs alone,
  // [30] a mixed burst (port forwarding and masquerade) that cannot run its
  // port-forwarding connections beside the split (dp_nat_mark, dp_nat_cross),
  // [31] a mixed burst's bound on the slots its inserts may add (dp_nat_prep),
  // [32] its creations' reverse keys registered, [33] masquerading records
  // dp_nat_cross looked up, [34] of them found (test counters).  The
  // allocating lane's bulk serve (dp_nat_lane, dp_nat_lane_assign): [35] the
  // lane records it served (the steps start after them), [36] the largest set
  // an allocating record asks + 1, [37] the complement of the smallest, [38]
  // an allocating record whose checks fail whatever the tuple or whose
  // reverse key may equal its initial key (no bulk serve), [39] the blocks it
  // logged
  unsigned long long *grp_tab, *grp_head, *grp_next;
  uint32_t *grp_list;
  uint32_t grp_mask;
  uint32_t burst;       // this burst's tag (never 0): entries of other bursts are empty
  // keyed index of the replaced fills: (burst, slot, old state, pf_repl index)
  uint4 *repl;
  uint32_t rmask;
  uint32_t force_seq;   // test hook (dpf_debug_nat_sequential): 1 the one-lane NAT pass always,
                        // 2 the split pass with every allocation on the lane alone (no wave batches),
                        // 3 no mode 4, 4 no mode 5 (a mixed burst on one lane), 5 the
                        // allocating lane without its bulk serve (every allocation in its steps),
                        // 6 its bulk serve with every block opened by one lane
  // the masquerading burst's allocating lane: its packets (bitmap by packet
  // index + summary, as pf_bits) and their order
  uint32_t *lane_bits, *lane_sum, *lane_order;
  uint4 *lane_plan;     // per lane record: its class and plan (dp_nat_lane_plan, 128 B)
  uint4 *lane_res;      // per lane record: its allocation for dp_nat_pairs (32 B)
  uint4 *lane_key;      // per lane record: what the lane's allocation step reads of its plan (48 B)
  // per record, a bit: dp_nat_mark found it a steady refresh (pfw::masq_steady_v)
  // as the burst started -- dp_nat_prep resolves it in place unless its flow
  // was tagged for the burst (a tag reaches both flows of a pair at once)
  unsigned long long *steady;
  unsigned long long *dup_tab;  // (burst << 32 | initial key hash) of the lane's allocating records
  // port forwarding near the capacity (mode 4): per record the new slots its
  // creation adds, then the sum of those of the records before it in packet
  // order (the table length its first insert meets); per 4096 records a sum
  uint32_t *adm, *adm_blk;
  uint32_t lean;        // the launch runs the flows variant without stateful NAT (dp_kernel.hip DP_SNAT)
  uint32_t ctx;         // the image's context tables fit the LDS copy (Image.ctx_bytes; the full units 15 / 16)
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
  uint32_t slot_tag;    // its flow's state word at attach (a refill by dp_nat_resolve changes it)
};

// the keyed index of the fills a burst's NAT pass replaced (FlowCtx::repl)
__host__ __device__ inline uint32_t repl_hash(uint32_t slot, uint32_t state) {
  uint32_t h = slot * 0x9E3779B1u ^ (state + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  return h ^ (h >> 12);
}

__host__ __device__ inline uint64_t make_ref(uint32_t slot, uint32_t state) {
  return ((uint64_t)(state >> 2) << 32) | slot;
}

}  // namespace dpf

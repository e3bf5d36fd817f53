// SPDX-License-Identifier: Apache-2.0
//
// Device table image layout (HBM).  Produced by the host table compiler
// (dp_tables.cpp) from the lowered descriptors of include/dpgpu.h, consumed
// by the pipeline kernel (dp_kernel.hip).  One contiguous allocation; every
// "ptr" below is a byte offset from the image base, fixed up to a device
// pointer by the runtime before launch.
//
// Structures (see DESIGN.md "Data layout in HBM"):
//  - open-addressing hash maps (VNI -> FIB, VRF -> FIB, ifindex -> iface,
//    (ifindex, ip) -> adjacency MAC, classifier group keys, NAT table keys)
//  - per-FIB Poptrie-style LPM (direct-pointing table + 6-bit stride nodes
//    with popcount-compressed child/leaf arrays) for v4 and v6
//  - classifier = per-(vni_a, vni_b, gate) group bit-vector classifier
//    (Lakshman-Stiliadis): per-field elementary-interval index -> rule
//    bit-vector rows, ANDed word by word behind a summary (ABV) level;
//    first set bit = first match in precedence order
//  - static NAT = per-table elementary-interval index over NAT prefixes ->
//    longest covering entry, parent chain for shorter covers, sorted ranges
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

#define DPD_MAX_INSTR 4
// partial DoneReason histograms per context (kernel atomics spread over slots)
#define DPD_STAT_SLOTS 256

namespace dpd {

struct HashSlot {      // generic 16-byte open-addressing slot
  uint32_t k0, k1, k2; // key words; k2 bit31 = occupied
  uint32_t val;
};

struct HashMap {
  uint64_t slots;      // offset of HashSlot[mask+1]
  uint32_t mask;       // capacity - 1 (power of two), 0 if empty map
  uint32_t count;
};

// Poptrie node (6-bit stride): children bitmap + leaf-run bitmap
struct PtNode {
  uint64_t vec;        // bit v: slot v has a child node
  uint64_t leafvec;    // bit v: slot v starts a leaf run (non-child slots)
  uint32_t base1;      // first child node index
  uint32_t base0;      // first leaf index
  uint64_t pad;
};

#define DPD_LPM_D16 0x100u
struct Lpm {
  uint64_t direct;     // offset of uint32_t[1 << dbits]; bit31 = leaf(nh) else node idx
  uint32_t dbits;      // direct-pointing bits (16..24); | DPD_LPM_D16: DIR-24-8 with 16-bit
                       // direct entries (bit 15 leaf, else the block)
  uint32_t width;      // 32 or 128
  uint64_t blocks;     // != 0: DIR-24-8 -- a non-leaf direct entry is the index of a
                       // uint16_t[256] block of next hops for the last 8 bits (v4 with a
                       // 24-bit direct table); 0: Poptrie nodes below the direct table
  // v6 window (wtab != 0): the routes longer than /16 share their top wbits
  // bits (wpfx = those bits); a key inside that prefix reads
  // wtab[the wtb bits after them] -- leaf, or a Poptrie node at bit wbits + wtb
  // -- instead of walking the Poptrie down from bit 16
  uint64_t wtab;       // offset of uint32_t[1 << wtb]
  uint64_t wpfx;
  uint32_t wbits;      // 24..48
  uint32_t wtb;        // window table bits (wtab holds 2^wtb entries)
};

struct FibRec {
  uint32_t vrf_id;
  uint32_t flags;      // dp_fib_flag
  uint8_t vtep_fam;
  uint8_t vtep_mac[6];
  uint8_t pad0;
  uint8_t vtep_ip[16];
  Lpm v4, v6;
};

// Egress outcome resolved at publish time (Egress::egress_process depends
// only on (oif, next hop) and the interface / adjacency tables, which are
// part of the same immutable generation).
#define DPD_EG_NEED_ADJ 254u   // no next-hop address: adjacency of the packet's dst at run time

struct Instr {         // compacted dp_instr_t + resolved egress (64 B)
  uint8_t kind, flags, fam;
  uint8_t eg_code;     // EGRESS: DoneReason of Egress (DELIVERED = ok) or DPD_EG_NEED_ADJ
  uint32_t ifindex;
  uint32_t vni;
  uint8_t mac[6];
  uint8_t if_code;     // EGRESS: oif checks alone (255 = ok); used with DPD_EG_NEED_ADJ
  uint8_t pad2;
  uint8_t addr[16];
  uint64_t eg_dmac;    // adjacency MAC (48-bit, first byte most significant)
  uint64_t eg_smac;    // oif MAC
  uint64_t pad3;
};

struct Entry {
  uint32_t first_instr, n_instr;
};

struct RouteNh {
  uint32_t first_entry, n_entries;
};

// Resolved next hop, one per RouteNh (the values of the LPM leaves).  A route
// whose only FibEntry is a single Egress (or Drop) instruction is resolved in
// place, so the leaf reaches the egress outcome in one dependent load; any
// other route (ECMP, Local / decap, VXLAN encap, instruction lists) keeps the
// RouteNh -> Entry -> Instr chain (DPD_NH_CHAIN).
#define DPD_NH_CHAIN 0
#define DPD_NH_EGRESS 1
#define DPD_NH_DROP 2
struct alignas(16) NhRec {  // 32 B
  uint8_t kind, eg_code, if_code, has_oif;
  uint32_t oif;
  uint32_t entry;      // FibEntry index (EGRESS / DROP); CHAIN: first_entry
  uint32_t n_entries;  // CHAIN
  uint64_t eg_dmac, eg_smac;
};
static_assert(sizeof(NhRec) == 32, "NhRec is 32 B");

// Interface record with Ingress's table-only checks pre-evaluated
// (dataplane/src/packet_processor/ingress.rs:153-182)
struct IfRec {         // 32 B
  uint32_t ifindex;
  uint8_t valid;       // 0: no such interface (InterfaceUnknown)
  uint8_t pre_code;    // admin down / unsupported type, checked before the MAC (255 = ok)
  uint8_t post_code;   // attach: bridge -> Unsupported, none -> Detached (255 = VRF)
  uint8_t pad;
  uint32_t vrf_id;
  int32_t fib;         // FIB of vrf_id (-1: none -> InternalFailure in IP-Forward)
  uint64_t mac;        // 48-bit
  uint64_t pad2;
};

// Multibit index descriptor (see FieldIdx / NatTab) copied into the context
// record that leads to the index, so the hot path walks it without first
// loading the Group / NatTab record (one dependent load less per lookup).
struct Mbi {           // 16 B (image offsets < 4 GiB: dp_tables.cpp refuses larger images)
  uint32_t root;       // 0: not usable here (bit-vector group, bounds form, absent table)
  uint32_t blocks;
  uint8_t s0, kbits;   // root stride, key width (32 address / 16 port)
  uint8_t field;       // classifier: the indexed field (0 src, 1 dst, 2 sport, 3 dport)
  uint8_t pad;
  uint32_t pad2;
};
static_assert(sizeof(Mbi) == 16, "Mbi is 16 B");

// Per source VNI context.  The records are the open-addressing slots of the
// VNI map themselves (key `vni`, 0 = empty: VNI 0 is invalid,
// net/src/vxlan/vni.rs:76-82), so one dependent load finds the context.
struct alignas(16) VniRec {  // 96 B
  uint32_t vni;
  uint32_t fib;        // FIB index of the VNI
  uint32_t vrf_id;
  int32_t ffr[2];      // flow-filter remote group (vni, 0, 0) v4 / v6, -1
  int32_t nat_dst;     // NAT dst table of the VNI's PerVniTable, -1
  uint32_t pervni;     // a PerVniTable exists for the VNI
  uint32_t pad;
  Mbi ffr4;            // index of the v4 remote group (candidate-list form)
  Mbi ndst;            // index of the NAT dst table
  uint64_t pad2[4];
};
static_assert(sizeof(VniRec) == 96, "VniRec is 96 B");

// Per (src VNI, dst VNI) context: target of a flow-filter remote verdict
struct alignas(16) PairRec {  // 128 B
  int32_t ffl[2];      // flow-filter local group (src, dst, 0) v4 / v6
  int32_t acl[2];      // ACL group (src, dst, 0) v4 / v6
  uint32_t acl_def;    // default action + 1, 0 = none
  int32_t nat_src;     // NAT src table (src -> dst), -1
  int32_t dst_fib;     // FIB of the dst VNI, -1
  uint32_t dst_vni;
  Mbi ffl4;            // index of the v4 local group (candidate-list form)
  Mbi acl4;            // index of the v4 ACL group (candidate-list form)
  Mbi acl4b;           // the ACL group's second list index (Group.lfield2), root 0: none
  Mbi nsrc;            // index of the NAT src table
  uint64_t lpm4_direct;  // the dst FIB's v4 LPM (Lpm.direct / dbits / blocks), 0: none
  uint32_t lpm4_dbits;
  uint32_t pad;
  uint64_t lpm4_blocks;
  uint64_t pad2;
};
static_assert(sizeof(PairRec) == 128, "PairRec is 128 B");

struct Adj {           // adjacency slot (open addressing, keyed ifindex+ip)
  uint32_t ifindex;
  uint8_t fam, used, pad[2];
  uint8_t addr[16];
  uint8_t mac[6];
  uint8_t pad2[2];
};

struct AdjMap {
  uint64_t slots;      // Adj[mask+1]
  uint32_t mask;
  uint32_t count;
};

// --- classifier -----------------------------------------------------------
// Field order: 0 src ip, 1 dst ip, 2 sport, 3 dport.  Keys are 128-bit
// (hi, lo); v4 addresses and ports use hi = 0.
// Elementary-interval index of one field.  Two forms:
//  - multibit table (v4 addresses, ports; root != 0): root[key >> (kbits - s0)]
//    then 8-bit blocks; an entry with bit 31 set is the interval's row id,
//    otherwise the index of the next 256-entry block (<= 3 more levels);
//  - sorted bounds (v6, or few intervals): binary search, narrowed by an
//    optional 16-bit jump table, then rows[interval].
#define DPD_LEAF 0x80000000u
struct FieldIdx {
  uint64_t bounds;     // offset of uint64_t[2*n] (hi, lo) interval starts, ascending
  uint64_t rows;       // offset of uint32_t[n] row index per interval
  uint64_t jump;       // offset of uint32_t[65537]: interval containing the start of
                       // each 16-bit top-bits bucket (0: no jump table, n small)
  uint64_t root;       // multibit root uint32_t[1 << s0] (0: bounds form)
  uint64_t blocks;     // multibit blocks uint32_t[256 * k]
  uint32_t n;          // number of intervals (>= 1; bounds[0] = 0)
  uint8_t shift;       // key >> shift = bucket (v4 ip: 16, port: 0, v6: hi >> 48)
  uint8_t s0;          // multibit root stride (bits)
  uint8_t kbits;       // multibit key width (32 or 16)
  uint8_t pad;
};

// Candidate-list form of a group (mode DPD_GROUP_LIST): one field (`lfield`)
// is indexed; its elementary interval maps to a run of CandRec -- the
// group's rules whose `lfield` range covers the interval, in precedence
// order, stored inline with every field and the rule's actions.  A lookup
// reads the index, then verifies candidates in order until the first full
// match: a few cache lines per packet instead of one bit-vector row per
// field.  The table compiler chooses it when every list is short
// (dp_tables.cpp build_classifier) and keeps the bit-vector form otherwise.
// Index leaves (multibit DPD_LEAF entries, or rows[] of the bounds form)
// hold a packed run: first record << DPD_RUN_BITS | count.
#define DPD_GROUP_BV 0
#define DPD_GROUP_LIST 1
#define DPD_NO_FIELD 0xffu
#define DPD_RUN_BITS 6
#define DPD_RUN_MAX 63
struct CandRec {       // 64 B, 64-byte aligned: one sector per candidate
  uint64_t src_hi, src_lo;   // prefix network, key form (v4: hi 0, lo addr)
  uint64_t dst_hi, dst_lo;
  uint8_t slen, dlen;        // prefix lengths (v4: of 32, v6: of 128)
  uint8_t proto_val, proto_mask;
  uint16_t sp_lo, sp_hi, dp_lo, dp_hi;
  uint32_t rule;             // global rule index (table's rule arrays)
  uint32_t action, action2, aux, orig;
};
static_assert(sizeof(CandRec) == 64, "CandRec is one 64-byte sector");
// v4 candidate (32 B, two per sector): the predicates plus the three action
// words a v4 lookup reads.  act0 = action; act1 = action2 (flow-filter
// remote) or the caller's rule index (ACL, flow-filter local); act2 = the
// PairRec index (flow-filter remote) or the global rule index.
struct alignas(16) CandRec4 {
  uint32_t src, dst;                   // prefix networks
  uint8_t slen, dlen, proto_val, proto_mask;
  uint16_t sp_lo, sp_hi;
  uint16_t dp_lo, dp_hi;
  uint32_t act0, act1, act2;
};
static_assert(sizeof(CandRec4) == 32, "CandRec4 is 32 B");

struct Group {
  uint32_t n_rules;
  uint32_t words;      // W = ceil(n_rules / 64)
  uint32_t sum_words;  // S = ceil(W / 64)
  uint32_t rule_base;  // index of rule 0 of this group in the table's rule arrays
  uint32_t mode;       // DPD_GROUP_BV / DPD_GROUP_LIST
  uint32_t lfield;     // LIST: the indexed field (0 src, 1 dst, 2 sport, 3 dport)
  uint32_t lfield2;    // LIST: a second indexed field (DPD_NO_FIELD: none); its runs hold
                       // the same candidates for the other field's intervals, so a lookup
                       // may verify whichever of the two runs is shorter
  uint32_t pad_l;
  uint64_t recs;       // LIST: offset of CandRec[]
  uint64_t pool;       // BV: offset of uint64_t rows[row][S + W]
  uint64_t proto_rows; // BV: offset of uint16_t[256]
  FieldIdx f[4];
};

struct Classifier {
  HashMap groups;      // (vni_a, vni_b, gate) -> group index (host side / fallback)
  uint64_t group_recs; // Group[]
  uint64_t action;     // uint32_t[n_rules_total]
  uint64_t action2;    // uint32_t[n_rules_total]
  uint64_t orig;       // uint32_t[n_rules_total] (index in the caller's array)
  uint64_t aux;        // uint32_t[n_rules_total]: flow-filter remote -> PairRec index
  uint64_t recs;       // candidate records of the list groups (shared by all groups):
                       // CandRec4[] in a v4 classifier, CandRec[] in a v6 one
  uint32_t n_groups;
  uint32_t n_rules;
};

// --- static NAT ------------------------------------------------------------
struct NatRange {
  uint32_t olo_ip, ohi_ip;   // host order
  uint16_t olo_port, ohi_port;
  uint32_t tlo_ip, thi_ip;
  uint16_t tlo_port, thi_port;
  uint32_t pad;
  uint64_t offset;
};

// 64 B, one sector: the entry plus an inline copy of its range when it has
// exactly one (the common case: the lookup then needs no range search).
struct alignas(16) NatEnt {
  uint32_t net;              // prefix network (host order)
  // inl: bit 0 the range is inline (n_ranges == 1, offset < 2^32), bit 1
  // the port range is (n_pr == 1: first_pr holds it, packed)
  uint8_t len, is_pat, covers_all, inl;
  int32_t parent;            // next shorter covering entry in this table, -1
  uint32_t first_pr, n_pr;   // uint32_t packed (lo | hi<<16)
  uint32_t first_range, n_ranges;
  uint32_t size_lo, size_hi; // Nat: ip_len(); Pat: size()
  uint32_t olo_ip, ohi_ip;   // inline range (NatRange fields)
  uint16_t olo_port, ohi_port;
  uint32_t tlo_ip, thi_ip;
  uint16_t tlo_port, thi_port;
  uint32_t offset;
};
static_assert(sizeof(NatEnt) == 64, "NatEnt is one 64-byte sector");

struct NatTab {
  uint64_t bounds;           // uint32_t[n] interval starts (host order)
  uint64_t longest;          // int32_t[n] longest covering entry (global idx) or -1
  uint64_t root;             // multibit table (0: bounds form); leaf = DPD_LEAF | (entry + 1)
  uint64_t blocks;
  uint32_t n;
  uint8_t s0;                // root stride (16, or 8 for configurations with many tables)
  uint8_t pad[3];
};

// A port-forwarding entry (PortFwEntry, nat/src/portfw/portfwtable/
// objects.rs:30-39) with its id (the identity its Weak refs name).
struct PfRuleRec {
  uint32_t id;
  uint32_t src_vni, dst_vni;
  uint8_t proto, fam, plen, pad;
  uint16_t ext_lo, ext_hi, int_lo, int_hi;
  uint32_t ext[4], inn[4];       // networks, big-endian words (v4: word 0)
  uint64_t init_ns, estab_ns;    // init_timeout / estab_timeout
};

struct Image {
  uint64_t bytes;
  int64_t genid;
  uint64_t vni_slots;        // VniRec[vni_mask + 1], open addressing on hmix(vni, 0, 0)
  uint32_t vni_mask;
  uint32_t pad_vni;
  HashMap vrf_fib;           // vrf id -> fib index
  uint64_t fibs;             // FibRec[]
  uint32_t n_fibs;
  uint32_t drop_nh;          // route nh of the default /0 drop route
  uint64_t pt_nodes;         // PtNode[]
  uint64_t pt_leaves;        // uint32_t[]
  uint64_t route_nhs;        // RouteNh[]
  uint64_t nh_recs;          // NhRec[] (parallel to route_nhs)
  uint64_t entries;          // Entry[]
  uint64_t instrs;           // Instr[]
  HashMap ifaces;            // ifindex -> IfRec index
  uint64_t if_recs;          // IfRec[]
  uint64_t if_direct;        // IfRec[if_direct_n], indexed by ifindex (small ifindexes)
  uint32_t if_direct_n;
  uint32_t n_vni_recs;
  HashMap pairs;             // (src vni, dst vni) -> PairRec index
  uint64_t pair_recs;        // PairRec[]
  AdjMap adjs;
  Classifier acl[2];         // [0] v4, [1] v6
  HashMap acl_default;       // (src_vni, dst_vni) -> action + 1
  Classifier ff_remote[2];
  Classifier ff_local[2];
  HashMap nat_tabs;          // (kind, src_vni, dst_vni) -> NatTab index
  HashMap nat_pervni;        // src_vni -> 1 (PerVniTable exists)
  uint64_t nat_tab_recs;     // NatTab[]
  uint64_t nat_ents;         // NatEnt[]
  uint64_t nat_prs;          // uint32_t[]
  uint64_t nat_ranges;       // NatRange[]
  // port forwarding: (src_vni, proto) -> run of PfRuleRec sorted by prefix
  // length, longest first (val = first << 16 | count); entry id -> index
  HashMap pf_keys;
  HashMap pf_ids;
  uint64_t pf_rules;         // PfRuleRec[]
  uint32_t n_pf;
  uint32_t may_encap;        // some FibEntry encapsulates: an output may start before its frame
  // v6 window of the classifiers' v6 address indexes (0: none): every v6
  // rule prefix lies inside one prefix of v6w_c bits (value v6w_p), and the
  // bounds and jump tables of v6 address fields are over the key transformed
  // by v6_window_key (dp_kernel.hip): 0 below it, all ones above it, else the
  // key shifted left by v6w_c with bit 0 set
  uint32_t v6w_c;
  uint32_t v6w_fib;  // 1: some v6 FIB has a window table (Lpm.wtab)
  uint64_t v6w_p;
  // 1: the image configures stateful NAT -- a flow-filter rule requiring port
  // forwarding or masquerade, a port-forwarding rule or a masquerade expose
  // (the flows variant without that code serves tables that never held it)
  uint32_t snat;
  // 1: the image configures masquerade (a flow-filter rule requiring it or a
  // masquerade expose): a flows burst sizes the masquerade split's lane
  // scratch (dp_runtime.cpp)
  uint32_t masq;
  // 1: two port-forwarding rules may map onto one internal address and port
  // (their internal sides overlap): a creation's reverse key may then be a
  // flow of another connection's pair (dp_nat_mark probes for it)
  uint32_t pf_overlap;
  uint32_t n_nh;             // NhRec count
  // The context tables every packet reads -- VNI slots, the pair map's slots,
  // PairRecs, NhRecs -- copied into each workgroup's LDS when together they
  // fit DPD_CTX_MAX (ctx_bytes > 0; 0: read from HBM): VNI slots at 0, then
  // the others at these offsets (16-byte aligned)
  uint32_t n_pair_recs;
  uint32_t ctx_bytes;
  uint32_t ctx_pslots, ctx_prec, ctx_nh;
};
constexpr uint32_t DPD_CTX_MAX = 7168;

// 32-bit mixing hash for the open-addressing maps (host and device agree)
__host__ __device__ inline uint32_t hmix(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u;
  h ^= (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

}  // namespace dpd

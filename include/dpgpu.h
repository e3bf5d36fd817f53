/* SPDX-License-Identifier: Apache-2.0
 *
 * dpgpu.h -- C ABI of the MI355X (gfx950) per-burst packet path.
 *
 * This is the drop-in boundary for the reference's packet hot loop
 * (githedgehog/dataplane).  The reference composes the path from NetworkFunction
 * stages (pipeline/src/static_nf.rs:12-32) assembled in
 * dataplane/src/packet_processor/mod.rs:130-145:
 *
 *   Ingress -> IP-Forward-1 -> IcmpErrorHandler -> FlowLookup -> FlowFilter ->
 *   AclFilter -> StaticNat -> PortForwarder -> Masquerade -> IP-Forward-2 -> Egress
 *
 * followed by Packet::serialize (net/src/packet/mod.rs:363-374).  One call of
 * dp_process_burst*() runs that whole block for a burst, on the GPU.  The
 * FlowTable FlowLookup and IcmpErrorHandler consult is a device flow table
 * attached to the context (dp_ctx_attach_flow_table; none attached = an
 * empty table).  PortForwarder runs on the GPU over the
 * port-forwarding rules of the tables (dp_portfw_rule_t) and creates its flow
 * pairs in the attached flow table; Masquerade runs on the GPU over the
 * masquerade exposes (dp_masq_expose_t) with its port allocator as device
 * state of the attached flow table.  AclFilter's classifier is also callable
 * alone (dp_acl_classify: the batch Lookup of acl/src/dpdk/lookup.rs).
 *
 * A Rust `GpuPathNf: NetworkFunction` materialises the burst
 * exactly like FlowFilter::process does (flow-filter/src/lib.rs:357-362),
 * stages the frames + metadata into the buffers below, calls this ABI and
 * applies the returned DoneReason / metadata to each Packet.
 *
 * Conventions
 *  - Every function returns 0 on success or a negative errno value.  Per-packet
 *    failures are never status codes: they are DoneReason values in dp_pkt_out_t
 *    (net/src/packet/meta.rs:84-119).  A whole-burst failure marks every packet
 *    DP_DONE_INTERNAL_FAILURE, as the reference stages do for unreadable tables
 *    (dataplane/src/packet_processor/ipforward.rs:89-98).
 *  - Addresses, MACs and prefixes are in network byte order.
 *  - The library never retains caller memory past a call.
 *  - A context is used by one thread (one dp-worker); dp_tables_publish may be
 *    called from another thread (mgmt) and only swaps a pointer for bursts
 *    that start after it returns (left-right / ArcSwap semantics,
 *    routing/src/fib/fibtype.rs:323-392, flow-filter/src/context/mod.rs:40-90).
 */
#ifndef DPGPU_H
#define DPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPGPU_ABI_VERSION 7u

/* Bytes every frame must have in front of it (its own scratch, owned by the
 * packet).  Output headers are written in place into this headroom: VXLAN
 * encap over an IPv6 underlay grows the frame by at most 14+40+8+8 = 70 B.
 * Mirrors TestBuffer's 96 B headroom (net/src/buffer/test_buffer.rs:45-50). */
#define DP_HEADROOM 96u

/* ------------------------------------------------------------------------ */
/* DoneReason, in the reference's declaration order (u8 ordinals),           */
/* net/src/packet/meta.rs:84-119.                                            */
/* ------------------------------------------------------------------------ */
enum dp_done_reason {
    DP_DONE_INTERNAL_FAILURE = 0,
    DP_DONE_INTERFACE_UNKNOWN = 1,
    DP_DONE_INTERFACE_DETACHED = 2,
    DP_DONE_INTERFACE_ADM_DOWN = 3,
    DP_DONE_INTERFACE_OPER_DOWN = 4,
    DP_DONE_INTERFACE_UNSUPPORTED = 5,
    DP_DONE_NOT_ETHERNET = 6,
    DP_DONE_UNHANDLED = 7,
    DP_DONE_MAC_NOT_FOR_US = 8,
    DP_DONE_INVALID_DST_MAC = 9,
    DP_DONE_MISSING_ETHER_TYPE = 10,
    DP_DONE_NOT_IP = 11,
    DP_DONE_ROUTE_FAILURE = 12,
    DP_DONE_ROUTE_DROP = 13,
    DP_DONE_HOP_LIMIT_EXCEEDED = 14,
    DP_DONE_MISS_L2_RESOLUTION = 15,
    DP_DONE_VXLAN_DECAP_FAILURE = 16,
    DP_DONE_VXLAN_ENCAP_FAILURE = 17,
    DP_DONE_FILTERED = 18,
    DP_DONE_ACL_DROPPED = 19,
    DP_DONE_NAT_OUT_OF_RESOURCES = 20,
    DP_DONE_FLOW_CAPACITY_EXCEEDED = 21,
    DP_DONE_NAT_UNSUPPORTED_PROTO = 22,
    DP_DONE_NAT_FAILURE = 23,
    DP_DONE_NAT_NOT_PORT_FORWARDED = 24,
    DP_DONE_MALFORMED = 25,
    DP_DONE_UNROUTABLE = 26,
    DP_DONE_INVALID_CHECKSUM = 27,
    DP_DONE_ICMP_ERROR_INCOMPLETE = 28,
    DP_DONE_INTERNAL_DROP = 29,
    DP_DONE_LOCAL = 30,
    DP_DONE_DELIVERED = 31,
    DP_DONE_DEPARSE_ERROR = 32,
    DP_DONE_NO_HEAD_ROOM = 33,
    DP_DONE_COUNT = 34,
    /* "not done": only ever seen if a stage sequence leaves a packet pending,
     * which the router pipeline never does (Egress always decides). */
    DP_DONE_NONE = 255
};

/* PacketMeta flags, bit-identical to MetaFlags (net/src/packet/meta.rs:121-136). */
enum dp_meta_flag {
    DP_META_INITIALIZED = 1u << 0,
    DP_META_IS_L2_BCAST = 1u << 1,
    DP_META_NATTED_SRC = 1u << 2,
    DP_META_NATTED_DST = 1u << 3,
    DP_META_REFR_CHKSUM = 1u << 4,
    DP_META_KEEP = 1u << 5,
    DP_META_IS_OVERLAY = 1u << 6,
    DP_META_REQ_MASQUERADE = 1u << 7,
    DP_META_REQ_PORT_FORWARDING = 1u << 8,
    DP_META_REQ_STATIC_NAT_SRC = 1u << 9,
    DP_META_REQ_STATIC_NAT_DST = 1u << 10
};

/* ------------------------------------------------------------------------ */
/* Burst descriptors (SoA-friendly fixed-size records, 16 B in / 32 B out).  */
/* ------------------------------------------------------------------------ */

/* dp_pkt_in_t.flags */
enum dp_in_flag {
    /* Harness idiom of nat/src/static_nat/test.rs:285-296 and
     * flow-filter tests: the frame is the INNER frame of a VXLAN packet that
     * IP-Forward-1 has already decapsulated.  src_vni is the VNI it arrived
     * on; Ingress and IP-Forward-1 are skipped and the metadata is set exactly
     * as packet_exec_instruction_local sets it after a successful decap
     * (dataplane/src/packet_processor/ipforward.rs:140-161): src_vpcd=VNI,
     * vrf=fib(VNI).id, IS_OVERLAY; an unregistered VNI gives Unroutable. */
    DP_IN_SEEDED_OVERLAY = 1u << 0
};

typedef struct dp_pkt_in {
    uint32_t off;      /* frame start inside the burst buffer; >= DP_HEADROOM
                          bytes in front of it belong to this packet */
    uint16_t len;      /* frame length (mbuf data_len, FCS stripped) */
    uint16_t flags;    /* enum dp_in_flag */
    uint32_t iif;      /* PacketMeta.iif, set by the driver */
    uint32_t src_vni;  /* only with DP_IN_SEEDED_OVERLAY */
} dp_pkt_in_t;

/* What the driver needs to transmit or drop a packet (16 B, always written). */
typedef struct dp_pkt_out {
    uint32_t off;        /* serialized frame start (only valid if Delivered) */
    uint16_t len;        /* serialized frame length (only valid if Delivered) */
    uint8_t done;        /* enum dp_done_reason */
    uint8_t acl;         /* 0: ACL not consulted, 1: allow (rule), 2: deny (rule),
                            3: allow (peering default), 4: deny (peering default),
                            5: allow (no ACL for peering), 6: allow (reply of a
                            flow a Flow-scope rule allowed; acl_rule = that rule) */
    uint32_t oif;        /* PacketMeta.oif (0 if None) */
    uint16_t meta_flags; /* enum dp_meta_flag (MetaFlags, 11 bits) */
    uint16_t pad;
} dp_pkt_out_t;

/* dp_pkt_meta_t.pm_flags: which Option<> fields of PacketMeta are Some */
enum dp_pm_flag {
    DP_PM_HAS_VRF = 1u << 0,   /* vrf */
    DP_PM_HAS_NH = 1u << 1,    /* nh_addr */
    DP_PM_HAS_DSCP = 1u << 2   /* dscp and ecn (set together, ipforward.rs:143-148) */
};

/* The rest of PacketMeta (net/src/packet/meta.rs:138-154), 48 B, written
 * only when the caller passes a meta array: the fields a CPU stage kept
 * after the GPU block (PacketStatsNF, per-VPC stats, a dumper) would read. */
typedef struct dp_pkt_meta {
    uint32_t dst_vni;    /* PacketMeta.dst_vpcd VNI (0 if None) */
    uint32_t src_vni;    /* PacketMeta.src_vpcd VNI (0 if None) */
    uint32_t fib_entry;  /* index of the last FibEntry executed (UINT32_MAX: none) */
    uint32_t acl_rule;   /* index of the matching ACL rule in its table (UINT32_MAX: none) */
    uint32_t vrf;        /* PacketMeta.vrf (DP_PM_HAS_VRF) */
    uint8_t pm_flags;    /* enum dp_pm_flag */
    uint8_t dscp;        /* PacketMeta.dscp (DP_PM_HAS_DSCP) */
    uint8_t ecn;         /* PacketMeta.ecn (DP_PM_HAS_DSCP) */
    uint8_t nh_family;   /* 4 / 6 (DP_PM_HAS_NH) */
    uint8_t nh_addr[16]; /* PacketMeta.nh_addr, network order (v4: first 4 bytes) */
    uint64_t flow_ref;   /* PacketMeta.flow_info as a flow-table ref (DP_FLOW_NONE: None) */
} dp_pkt_meta_t;

/* ------------------------------------------------------------------------ */
/* Table descriptors: host arrays lowered from the reference's structures.  */
/* ------------------------------------------------------------------------ */

typedef struct dp_ipaddr {
    uint8_t family;  /* 4 or 6 (0: none) */
    uint8_t pad[3];
    uint8_t addr[16]; /* v4 uses addr[0..4] */
} dp_ipaddr_t;

typedef struct dp_prefix {
    uint8_t family;  /* 4 or 6 */
    uint8_t len;     /* prefix length; host bits must be zero
                        (lpm/src/prefix/ip.rs:148-165) */
    uint8_t pad[2];
    uint8_t addr[16];
} dp_prefix_t;

/* FIB: routing/src/fib/fibtype.rs:54-61.  One per VRF. */
enum dp_fib_flag {
    DP_FIB_VTEP_HAS_IP = 1u << 0,
    DP_FIB_VTEP_HAS_MAC = 1u << 1
};
typedef struct dp_fib {
    uint32_t vrf_id;        /* FibKey::Id */
    uint32_t flags;         /* enum dp_fib_flag */
    dp_ipaddr_t vtep_ip;    /* Vtep (routing/src/evpn/vtep.rs:11-14) */
    uint8_t vtep_mac[6];
    uint8_t pad[2];
} dp_fib_t;

/* FibTable VNI registration (routing/src/fib/fibtable.rs:46-56). */
typedef struct dp_vni_fib {
    uint32_t vni;
    uint32_t fib;           /* index into fibs[] */
} dp_vni_fib_t;

/* PktInstruction (routing/src/fib/fibobjects.rs:258-264). */
enum dp_instr_kind {
    DP_INSTR_DROP = 0,
    DP_INSTR_LOCAL = 1,
    DP_INSTR_ENCAP_VXLAN = 2,
    DP_INSTR_EGRESS = 3
};
enum dp_instr_flag {
    DP_INSTR_HAS_IFINDEX = 1u << 0, /* EgressObject.ifindex is Some */
    DP_INSTR_HAS_ADDR = 1u << 1,    /* EgressObject.address is Some */
    DP_INSTR_HAS_DMAC = 1u << 2     /* VxlanEncapsulation.dmac is Some */
};
typedef struct dp_instr {
    uint32_t kind;          /* enum dp_instr_kind */
    uint32_t flags;         /* enum dp_instr_flag */
    uint32_t ifindex;       /* LOCAL / EGRESS */
    uint32_t vni;           /* ENCAP_VXLAN */
    dp_ipaddr_t addr;       /* EGRESS next-hop / ENCAP_VXLAN remote */
    uint8_t mac[6];         /* ENCAP_VXLAN dmac */
    uint8_t pad[2];
} dp_instr_t;

/* FibEntry = ordered instruction list (fibobjects.rs:142-144). */
typedef struct dp_fib_entry {
    uint32_t first_instr;
    uint32_t n_instr;       /* 1..4 */
} dp_fib_entry_t;

/* FibRoute = its FibGroups' entries, flattened in group order
 * (routing/src/fib/fibgroupstore.rs:195-234). */
typedef struct dp_route_nh {
    uint32_t first_entry;
    uint32_t n_entries;     /* >= 1; > 1 selects by packet_hash_ecmp */
} dp_route_nh_t;

typedef struct dp_route {
    dp_prefix_t prefix;
    uint32_t fib;           /* index into fibs[] */
    uint32_t nh;            /* index into route_nhs[] */
} dp_route_t;

/* Interface table (routing/src/interfaces/interface.rs). */
enum dp_if_state { DP_IF_UNKNOWN = 0, DP_IF_DOWN = 1, DP_IF_UP = 2 };
enum dp_if_type { DP_IFT_UNKNOWN = 0, DP_IFT_ETHERNET = 1, DP_IFT_DOT1Q = 2,
                  DP_IFT_LOOPBACK = 3, DP_IFT_VXLAN = 4 };
enum dp_if_attach { DP_ATTACH_NONE = 0, DP_ATTACH_VRF = 1, DP_ATTACH_BRIDGE = 2 };
typedef struct dp_iface {
    uint32_t ifindex;
    uint8_t admin_state;    /* enum dp_if_state */
    uint8_t oper_state;     /* enum dp_if_state */
    uint8_t iftype;         /* enum dp_if_type (Ethernet/Dot1q carry a MAC) */
    uint8_t attach;         /* enum dp_if_attach */
    uint32_t vrf_id;        /* Attachment::Vrf(fibkey) */
    uint8_t mac[6];
    uint8_t pad[2];
} dp_iface_t;

/* Adjacency table, keyed (ifindex, ip) (routing/src/atable/adjacency.rs:51-82). */
typedef struct dp_adjacency {
    dp_ipaddr_t addr;
    uint32_t ifindex;
    uint8_t mac[6];
    uint8_t pad[2];
} dp_adjacency_t;

/* Classifier rule: the union of the reference's three MatchKeys
 *   AclKey    (acl-filter/src/context.rs:168-190)
 *   RemoteKey (flow-filter/src/context/tables.rs:192-207)
 *   LocalKey  (flow-filter/src/context/tables.rs:211-229)
 * with match-action predicate semantics (match-action/src/predicate.rs):
 * proto = Mask, vni_a/vni_b/gate = Exact, src/dst = Prefix, ports = Range
 * (inclusive).  Unused fields are wildcards (prefix len 0, range 0..65535).
 *   ACL:       vni_a=src_vni, vni_b=dst_vni, gate=0
 *   FF remote: vni_a=src_vni, vni_b=GateVni (0 = ungated), src wildcard,
 *              sport wildcard
 *   FF local:  vni_a=src_vni, vni_b=dst_vni, gate=SourceGate, dst wildcard,
 *              dport wildcard */
typedef struct dp_rule {
    uint8_t proto_val;
    uint8_t proto_mask;     /* 0xff exact, 0x00 any */
    uint8_t family;         /* 4 or 6: which table */
    uint8_t gate;
    uint32_t vni_a;
    uint32_t vni_b;
    uint16_t sport_lo, sport_hi;
    uint16_t dport_lo, dport_hi;
    uint32_t priority;      /* flow-filter only: rule_priority(); tables are
                               matched in stable descending-priority order
                               (flow-filter/src/context/tables.rs:373-380);
                               ACL tables match in array order (first match,
                               acl-filter/src/context.rs:447-452) */
    dp_prefix_t src;
    dp_prefix_t dst;
    uint32_t action;        /* ACL: 0 Allow / 1 Deny.  FF remote: dst VNI.
                               FF local: enum dp_nat_mode (source NAT mode). */
    uint32_t action2;       /* FF remote: enum dp_nat_mode (destination NAT).
                               ACL: enum dp_acl_scope */
} dp_rule_t;

enum dp_acl_action { DP_ACL_ALLOW = 0, DP_ACL_DENY = 1 };
/* AclScope (config/src/external/overlay/acl.rs:137-141; Flow is the default):
 * a Flow-scope Allow also admits replies of a flow it allowed
 * (acl-filter/src/lib.rs:110-128). */
enum dp_acl_scope { DP_ACL_SCOPE_FLOW = 0, DP_ACL_SCOPE_PACKET = 1 };
/* NatRequirement (flow-filter/src/lib.rs NatMode = Option<NatRequirement>). */
enum dp_nat_mode { DP_NAT_NONE = 0, DP_NAT_STATIC = 1, DP_NAT_MASQUERADE = 2,
                   DP_NAT_PORT_FORWARDING = 3 };

/* Per-peering ACL default (acl-filter/src/context.rs:564-566). */
typedef struct dp_acl_default {
    uint32_t src_vni;
    uint32_t dst_vni;
    uint32_t action;        /* enum dp_acl_action */
} dp_acl_default_t;

/* Static NAT tables (nat/src/static_nat/setup/tables.rs), NAT44.
 * NatTables: src_vni -> PerVniTable{ dst_nat, src_nat[dst_vni] }. */
enum dp_nat_table_kind { DP_NAT_TABLE_DST = 0, DP_NAT_TABLE_SRC = 1 };
typedef struct dp_nat_table {
    uint32_t kind;          /* enum dp_nat_table_kind */
    uint32_t src_vni;       /* owning PerVniTable */
    uint32_t dst_vni;       /* DP_NAT_TABLE_SRC only: src_nat key */
    uint32_t first_entry;
    uint32_t n_entries;
} dp_nat_table_t;

/* One IpPortPrefixTrie entry: prefix -> NatTableValue. */
typedef struct dp_nat_entry {
    dp_prefix_t prefix;
    uint32_t is_pat;        /* NatTableValue::Pat (else ::Nat) */
    uint32_t first_port_range, n_port_ranges; /* Pat: prefix_port_ranges */
    uint32_t first_range, n_ranges;           /* ranges_tree, sorted by key */
    uint32_t pad;
    uint64_t size;          /* Nat: ip_len(); Pat: size() (ips x ports) */
} dp_nat_entry_t;

typedef struct dp_port_range {
    uint16_t lo, hi;        /* inclusive */
} dp_port_range_t;

/* ranges_tree element.  Nat:  key IpRange [orig_lo_ip, orig_hi_ip] ->
 * (target IpRange, offset).  Pat: key IpPortRangeBounds
 * [(orig_lo_ip,orig_lo_port), (orig_hi_ip,orig_hi_port)] ->
 * (IpPortRange{target ip range, target port range}, offset). */
typedef struct dp_nat_range {
    uint8_t orig_lo_ip[4];
    uint8_t orig_hi_ip[4];
    uint16_t orig_lo_port, orig_hi_port;
    uint8_t tgt_lo_ip[4];
    uint8_t tgt_hi_ip[4];
    uint16_t tgt_lo_port, tgt_hi_port;
    uint64_t offset;
} dp_nat_range_t;

/* Port-forwarding rule: PortFwEntry (nat/src/portfw/portfwtable/objects.rs:
 * 30-39, checks of PortFwEntry::new :70-155).  A publish applies the rule set
 * as PortFwTable::update does (:284-300): a rule that `matches` one of the
 * previous generation on the same device (same key, prefixes, port ranges and
 * destination VPC) is that same entry -- flows that refer to it stay valid
 * (their Weak upgrades) and only its timeouts change; rules no longer present
 * are gone; a new rule whose external range overlaps another of the same key
 * and external prefix is skipped (RangeSet overlap error, logged by the
 * reference).  Each entry has an id (dp_flow_info_t.pf_rule), stable while it
 * lives. */
typedef struct dp_portfw_rule {
    uint32_t src_vni;          /* PortFwKey.src_vpcd */
    uint8_t proto;             /* PortFwKey.proto: 6 (TCP) or 17 (UDP) */
    uint8_t pad[3];
    uint32_t dst_vni;          /* dst_vpcd (!= src_vni) */
    uint16_t ext_lo, ext_hi;   /* ext_ports: non-zero, ext_lo <= ext_hi */
    uint16_t int_lo, int_hi;   /* int_ports: same length */
    uint32_t init_timeout_s;   /* 0: PortFwEntry::DEFAULT_INITIAL_TOUT (10 s) */
    uint32_t estab_timeout_s;  /* 0: 30 min (TCP) / 30 s (UDP) */
    dp_prefix_t ext_prefix;    /* external prefix (what the client addresses) */
    dp_prefix_t int_prefix;    /* internal prefix (same family and length) */
} dp_portfw_rule_t;

/* Masquerade (stateful source NAT, nat/src/masquerade/).  One record per
 * masquerade expose of a stateful-NAT peering, in configuration order
 * (MasqueradeConfig::new, nat/src/masquerade/allocator_writer.rs:43-61;
 * gather_exposes, apalloc/setup.rs:95-137): the VPC whose private sources are
 * masqueraded towards the peer VPC, the expose's private prefixes (ips()),
 * its public ranges (as_range, the pools), its idle timeout, and the public
 * tuples the port-forwarding exposes of the same local manifest may claim
 * (claims_for, setup.rs:73-92), which the pools never hand out
 * (apalloc/reserved.rs).  An expose is one address family: its private and
 * public prefixes are all v4 (NAT44) or all v6 (NAT66).  Ports come in
 * bitmap order within a port block and addresses lowest first; the blocks of
 * an address come in index order (MasqueradeConfig::set_randomize(false), the
 * mode the reference's collision test runs, nat/src/masquerade/test.rs:
 * 1399-1406) or, with dp_tables_desc_t.masq_randomize, in a shuffled order
 * (the default, allocator_writer.rs:58; mgmt sets it, proc.rs:541): when an
 * address is put to use, its 256 blocks are permuted (PortAllocator::new,
 * port_alloc.rs:105-113).  The permutation is a function of masq_seed and
 * the address, so the device and any restatement agree:
 *   splitmix64(z): z += 0x9E3779B97F4A7C15; z = (z ^ z >> 30) * 0xBF58476D1CE4E5B9;
 *                  z = (z ^ z >> 27) * 0x94D049BB133111EB; return z ^ z >> 31
 *   x = masq_seed; for each 32-bit word w of the address as a 128-bit number,
 *   most significant first (v4: three zero words, then the address):
 *   x = splitmix64(x ^ w); perm = 0..255; for i = 255 down to 1:
 *   x = splitmix64(x); swap(perm[i], perm[x % (i + 1)])
 * and block i of the address covers ports [256 perm[i], 256 perm[i] + 255]. */
typedef struct dp_masq_expose {
    uint32_t src_vni;          /* MasqueradePeering.src_vpcd */
    uint32_t dst_vni;          /* MasqueradePeering.dst_vpcd */
    uint32_t idle_timeout_s;   /* expose idle_timeout (0: 120 s, setup.rs:25) */
    uint32_t first_prefix;     /* into masq_prefixes: n_private private prefixes,
                                  then n_public public ones */
    uint16_t n_private, n_public;
    uint32_t first_claim;      /* into masq_claims */
    uint32_t n_claims;
} dp_masq_expose_t;

/* A public (prefix, port range) a port-forwarding expose may claim, and the
 * L4 protocols of its rule (ExposeNat.proto). */
enum dp_masq_proto { DP_MASQ_TCP = 1u << 0, DP_MASQ_UDP = 1u << 1 };
typedef struct dp_masq_claim {
    dp_prefix_t prefix;
    uint16_t lo, hi;           /* inclusive */
    uint32_t protos;           /* enum dp_masq_proto */
} dp_masq_claim_t;

/* Addresses of one allocator region (a disjoint public range of one
 * protocol towards one peer VPC, apalloc/region.rs) that can be in use at
 * once: the region's lowest DP_MASQ_REGION_ADDRS offsets (the reference's
 * u32 offset bitmap, alloc.rs:349-377, bounded for device memory; each
 * address carries 64512 TCP / UDP ports). */
#define DP_MASQ_REGION_ADDRS 4096u
/* Addresses in use at once over one flow table's allocator (each carries its
 * PortAllocator, ~9 KiB of device memory): a new address past this many fails
 * as the region's exhaustion does (NoFreeIp; NoPoolFound when reserving). */
#define DP_MASQ_ADDRS 65536u

typedef struct dp_tables_desc {
    uint32_t abi_version;   /* DPGPU_ABI_VERSION */
    uint32_t pad0;
    int64_t genid;          /* PipelineData.genid (pipeline/src/pipeline.rs:22-42) */

    const dp_fib_t *fibs;            uint32_t n_fibs;
    const dp_vni_fib_t *vni_fibs;    uint32_t n_vni_fibs;
    const dp_route_t *routes;        uint64_t n_routes;
    const dp_route_nh_t *route_nhs;  uint32_t n_route_nhs;
    const dp_fib_entry_t *entries;   uint32_t n_entries;
    const dp_instr_t *instrs;        uint32_t n_instrs;
    const dp_iface_t *ifaces;        uint32_t n_ifaces;
    const dp_adjacency_t *adjs;      uint32_t n_adjs;

    const dp_rule_t *acl_v4;         uint32_t n_acl_v4;
    const dp_rule_t *acl_v6;         uint32_t n_acl_v6;
    const dp_acl_default_t *acl_defaults; uint32_t n_acl_defaults;

    const dp_rule_t *ff_remote_v4;   uint32_t n_ff_remote_v4;
    const dp_rule_t *ff_local_v4;    uint32_t n_ff_local_v4;
    const dp_rule_t *ff_remote_v6;   uint32_t n_ff_remote_v6;
    const dp_rule_t *ff_local_v6;    uint32_t n_ff_local_v6;

    const dp_nat_table_t *nat_tables; uint32_t n_nat_tables;
    const dp_nat_entry_t *nat_entries; uint32_t n_nat_entries;
    const dp_port_range_t *nat_port_ranges; uint32_t n_nat_port_ranges;
    const dp_nat_range_t *nat_ranges; uint32_t n_nat_ranges;

    const dp_portfw_rule_t *portfw;  uint32_t n_portfw;

    /* masquerade (NatAllocatorWriter::update_nat_allocator,
     * allocator_writer.rs:120-154, applied to the attached flow tables) */
    const dp_masq_expose_t *masq;    uint32_t n_masq;
    const dp_prefix_t *masq_prefixes; uint32_t n_masq_prefixes;
    const dp_masq_claim_t *masq_claims; uint32_t n_masq_claims;
    /* MasqueradeConfig identity: two generations with the same non-zero tag
     * are the same configuration (the allocator and its flows are kept, only
     * the generation advances); 0: compared by the exposes and claims above */
    uint64_t masq_config_tag;
    /* MasqueradeConfig::set_randomize (dp_masq_expose_t above): 1 shuffles
     * each address's port blocks by masq_seed; part of the configuration's
     * identity (a change rebuilds the allocators) */
    uint32_t masq_randomize;
    uint32_t pad1;
    uint64_t masq_seed;
} dp_tables_desc_t;

/* ------------------------------------------------------------------------ */
/* Errors (negative errno).                                                  */
/* ------------------------------------------------------------------------ */
#define DP_OK 0
#define DP_EINVAL (-22)
#define DP_ENOMEM (-12)
#define DP_ENODEV (-19)
#define DP_ENOTSUP (-95)   /* a table form the path does not support */
#define DP_EIO (-5)        /* HIP runtime failure */
#define DP_ENOTABLES (-61) /* no tables published yet (ENODATA) */

/* ------------------------------------------------------------------------ */
/* Entry points.                                                             */
/* ------------------------------------------------------------------------ */
typedef struct dp_ctx dp_ctx_t;

/* Library / ABI version (for the FFI loader's sanity check). */
uint32_t dp_abi_version(void);

/* One context per worker thread (worker.rs:175 builds one pipeline per
 * worker); owns one HIP stream and the device-side staging scratch.  Tables
 * are shared by all contexts on the same device (refcounted image). */
/* DP_ENOTSUP: the process maps two HIP runtimes (two copies of
 * libamdhip64 / libhsa-runtime64 -- e.g. PyTorch's bundled one loaded after
 * this library's); one runtime per process is required (DESIGN.md §5,
 * INTEGRATION.md §6). */
int dp_ctx_create(int device_ordinal, dp_ctx_t **out);
int dp_ctx_destroy(dp_ctx_t *ctx);

/* Compile the lowered tables into the device image and publish it.
 * Replaces left-right FibWriter publish / NatTablesWriter::update_nat_tables /
 * FlowFilterContextWriter::store / AclFilterContextWriter::store
 *  for every context on the device.  Never blocks a burst
 * beyond a pointer swap; the old image is retired once bursts using it end.
 * The attached flow tables' masquerade allocators follow the new
 * configuration within the call; if one cannot (device memory), the call
 * still publishes the tables, updates every other flow table, and returns the
 * first error -- the failed table tries again at its next burst, and that
 * burst fails whole (DP_DONE_INTERNAL_FAILURE) while it cannot. */
int dp_tables_publish(dp_ctx_t *ctx, const dp_tables_desc_t *tables);

/* Current generation id (PipelineData::genid). */
int64_t dp_tables_genid(const dp_ctx_t *ctx);

/* Host-origin burst: `buf` is caller-owned (pinned for best speed) host
 * memory holding every frame at in[i].off with DP_HEADROOM bytes in front.
 * Frames are rewritten in place; out[i] tells where each serialized frame
 * now starts; `meta` (may be NULL) receives the rest of each PacketMeta.
 * Synchronous.  `stats` (may be NULL) receives DP_DONE_COUNT
 * counters (PacketStatsNF, pipeline/src/sample_nfs.rs:225-273).  On any
 * error (layout violation, HIP failure) every out[i] is
 * DP_DONE_INTERNAL_FAILURE and the negative status is returned. */
int dp_process_burst(dp_ctx_t *ctx, uint8_t *buf, uint64_t buf_bytes,
                     const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta,
                     uint32_t n, uint64_t *stats);

/* Device-resident burst: every pointer is device memory; enqueued on
 * `stream` (a hipStream_t; NULL = the context's stream).  Asynchronous.
 * `dev_buf` must be 16-byte aligned and `buf_bytes` must cover every frame
 * end rounded up to 16 bytes (frames are staged with 16-byte loads); a
 * packet violating the layout contract is marked DP_DONE_INTERNAL_FAILURE
 * without touching memory, and a burst that cannot run at all (no tables,
 * misaligned buffer, launch failure) has every dev_out[i] marked
 * DP_DONE_INTERNAL_FAILURE on `stream` besides the negative status.
 * `dev_meta` (may be NULL: the bench path writes only the 16-byte out
 * records) receives the rest of each PacketMeta, flow_info included.
 * `dev_stats` (may be NULL) is accumulated into (DP_DONE_COUNT u64).
 * Bursts of one context may run concurrently on different streams. */
int dp_process_burst_device(dp_ctx_t *ctx, uint8_t *dev_buf, uint64_t buf_bytes,
                            const dp_pkt_in_t *dev_in, dp_pkt_out_t *dev_out,
                            dp_pkt_meta_t *dev_meta, uint32_t n, uint64_t *dev_stats,
                            void *stream);

/* Multi-GPU, host-origin burst: `ctxs` holds one
 * context per device (created by the caller, e.g. one per GPU of the node).
 * The burst -- laid out as for dp_process_burst, with packets in buffer
 * order and non-overlapping slots [off - DP_HEADROOM, off + len) -- is split
 * into n_ctx contiguous shards of whole packets (shard k: packets
 * [k n / n_ctx, (k+1) n / n_ctx)); each shard's byte span is copied to its
 * device with its own hipMemcpyAsync (every GPU has its own PCIe link, no
 * collective), processed there, and copied back.  Packets are independent,
 * so the result equals dp_process_burst on one device bit for bit
 * (tests/test_shard.py).  The analogue of the reference's per-worker fan-out
 * (dataplane/src/drivers/kernel/fanout.rs:49-73, worker.rs:175).
 * With a flow table: every context must be attached to the same one (else
 * DP_EINVAL) -- the reference's one Arc<FlowTable> shared by every worker --
 * and the shards are the workers' bursts, their flows launches run on the
 * table one after the other in shard order (one of the orders the
 * reference's concurrent workers may take): the result equals
 * dp_process_burst of each shard in turn on one context.  A flow table lives
 * on one device, so those contexts are contexts of one GPU.
 * Synchronous; `stats` (may be NULL) receives the summed DoneReason counts.
 * A whole-burst failure marks every packet DP_DONE_INTERNAL_FAILURE. */
int dp_process_burst_sharded(dp_ctx_t *const *ctxs, uint32_t n_ctx, uint8_t *buf,
                             uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                             dp_pkt_meta_t *meta, uint32_t n, uint64_t *stats);

/* Wait for the context's stream. */
int dp_ctx_synchronize(dp_ctx_t *ctx);

/* Context options (dp_ctx_set_option). */
enum dp_ctx_option {
    /* How dp_process_burst moves a host-origin burst:
     *   DP_HOST_AUTO      zero-copy when `buf`, `in` and `out` are all pinned,
     *                     device-mapped host memory (hipHostMalloc /
     *                     hipHostRegister) and `buf` is 16-byte aligned with
     *                     every frame end rounded up to 16 inside buf_bytes;
     *                     otherwise staged copies (default);
     *   DP_HOST_COPY      staged copies: each chunk's slot span and records
     *                     H2D, kernel, D2H, chunks overlapped on 3 streams;
     *   DP_HOST_ZERO_COPY zero-copy only: the kernel reads the frames and
     *                     records over PCIe and writes the rewritten header
     *                     spans and records back in place; a burst that does
     *                     not qualify fails with DP_EINVAL. */
    DP_OPT_HOST_PATH = 1,
    /* The flow clock (nanoseconds, the caller's clock -- the unit of
     * dp_flow_t.expires_at and dp_flow_sweep's `now`): Instant::now() for the
     * bursts that follow.  PortForwarder sets the expiry of the flows it
     * creates or refreshes to now + the rule's timeout
     * (flow_state.rs:233-263, flow_info.rs:399-407). */
    DP_OPT_CLOCK = 2
};
enum dp_host_path { DP_HOST_AUTO = 0, DP_HOST_COPY = 1, DP_HOST_ZERO_COPY = 2 };
int dp_ctx_set_option(dp_ctx_t *ctx, int option, int64_t value);

/* ------------------------------------------------------------------------ */
/* The ACL classifier alone (the narrower drop-in for A14):   */
/* AclFilter's classification as a batch lookup -- the reference's           */
/* Lookup<K, A> / DpdkAclLookup::lookup_batch (lookup/src/lib.rs:24-38,      */
/* acl/src/dpdk/lookup.rs:112-155), an rte_acl replacement.  Each key is     */
/* matched against the ACL of its (source VPC, destination VPC) peering in   */
/* the published tables: the first rule in rule order whose prefixes, ports  */
/* and protocol hold it, else the peering's default, else Allow              */
/* (acl-filter/src/lib.rs:96-137, acl/src/reference/table.rs:94-101).        */
/* ------------------------------------------------------------------------ */
typedef struct dp_acl_key {
    uint32_t src_vni, dst_vni;  /* the peering */
    uint8_t family;             /* 4 or 6 */
    uint8_t proto;              /* IP next header */
    uint16_t sport, dport;      /* 0 for a protocol without ports */
    uint8_t pad[2];
    uint8_t src[16], dst[16];   /* network byte order; v4 in the first 4 bytes */
} dp_acl_key_t;                 /* 48 B */

typedef struct dp_acl_result {
    uint32_t rule;    /* index of the matching rule in the published acl_v4 / acl_v6,
                         UINT32_MAX when none matched */
    uint8_t action;   /* enum dp_acl_action the key gets */
    uint8_t scope;    /* enum dp_acl_scope of the matching rule (0 without one) */
    uint8_t acl;      /* dp_pkt_out_t.acl's code: 1 / 2 rule allow / deny, 3 / 4 peering
                         default allow / deny, 5 no ACL for the peering; 0: a key of
                         another family than 4 / 6 (not classified) */
    uint8_t pad;
} dp_acl_result_t;    /* 8 B */

/* Classify n keys resident on the context's device into dev_out (stream as in
 * dp_process_burst_device; asynchronous there). */
int dp_acl_classify_device(dp_ctx_t *ctx, const dp_acl_key_t *dev_keys, dp_acl_result_t *dev_out,
                           uint32_t n, void *stream);
/* The same for keys and results in host memory (synchronous). */
int dp_acl_classify(dp_ctx_t *ctx, const dp_acl_key_t *keys, dp_acl_result_t *out, uint32_t n);

/* The reference's own key bytes.  AclKey<Ipv4Addr> / AclKey<Ipv6Addr>
 * (acl-filter/src/context.rs:168-190) as MatchKey::as_key_into writes them
 * (match-action-derive/src/lib.rs:191-206, 341-347): its fields back to back,
 * each big-endian (net/src/fixed_size.rs: NextHeader 1 byte, Vni right-aligned
 * in 4) -- proto, src_vni, dst_vni, src address, dst address, src port, dst
 * port: DP_ACL_MATCH_KEY_V4 (21) or DP_ACL_MATCH_KEY_V6 (45) bytes a key, the
 * key size naming the family.  Keys lie `stride` bytes apart (>= key_size;
 * lookup_batch's arena packs them at its layout's stride, lookup.rs:131-138),
 * so a binding hands over AclKey::as_key() output as it is.
 * dp_acl_key_from_match converts n of them to dp_acl_key_t (host code: no
 * device, no context); dp_acl_classify_match classifies them as
 * dp_acl_classify does.  DP_EINVAL: another key size, stride < key_size. */
#define DP_ACL_MATCH_KEY_V4 21u
#define DP_ACL_MATCH_KEY_V6 45u
int dp_acl_key_from_match(const uint8_t *match, uint32_t key_size, uint32_t stride, uint32_t n,
                          dp_acl_key_t *out);
int dp_acl_classify_match(dp_ctx_t *ctx, const uint8_t *match, uint32_t key_size, uint32_t stride,
                          uint32_t n, dp_acl_result_t *out);

/* ------------------------------------------------------------------------ */
/* The flow-filter classifier alone (the narrower drop-in for */
/* A13): FlowFilterContext::lookup_batch (flow-filter/src/context/tables.rs: */
/* 800-848) over the published ff_remote_* / ff_local_* rules.  Per input,   */
/* stage 1 matches the destination (RemoteKey: proto, src VNI, the GateVni   */
/* dst_vni -- 0 for an ungated lookup --, destination, destination port)     */
/* against the remote rules in priority order; on a hit, stage 2 matches the */
/* source (LocalKey: proto, src VNI, the verdict's VPC, source, source port, */
/* SourceGate) against the local rules (lookup_versioned, :854-915).  The    */
/* outcome is LookupResult (:70-81): Route (the verdict's VPC and NAT mode,  */
/* the source's NAT mode), SourceMiss (the verdict's VPC) or                 */
/* DestinationMiss -- also for an input whose two addresses are of different */
/* families.  Inputs are never reordered.                                   */
/* ------------------------------------------------------------------------ */
typedef struct dp_ff_input {        /* LookupInput (tables.rs:88-97) */
    uint32_t src_vni;               /* src_vpcd */
    uint32_t dst_vni;               /* dst_vpcd: stage 1's GateVni (0: None, an ungated lookup) */
    uint8_t src_family, dst_family; /* 4 or 6 each (IpAddr::V4 / V6) */
    uint8_t proto;                  /* NextHeader */
    uint8_t gate;                   /* SourceGate: 0 Ungated, 1 PortFwdReply */
    uint16_t sport, dport;          /* ports; None is (0, 0) */
    uint8_t pad[4];
    uint8_t src[16], dst[16];       /* network byte order; v4 in the first 4 bytes */
} dp_ff_input_t;                    /* 48 B */

enum dp_ff_outcome { DP_FF_DESTINATION_MISS = 0, DP_FF_SOURCE_MISS = 1, DP_FF_ROUTE = 2 };
typedef struct dp_ff_result {       /* LookupResult */
    uint8_t outcome;                /* enum dp_ff_outcome */
    uint8_t dst_nat;                /* Route: the verdict's NatMode (enum dp_nat_mode) */
    uint8_t src_nat;                /* Route: the source's NatMode */
    uint8_t pad;
    uint32_t dst_vni;               /* Route / SourceMiss: the verdict's dst_vpcd */
} dp_ff_result_t;                   /* 8 B */

/* n inputs resident on the context's device (stream as in
 * dp_process_burst_device; asynchronous there). */
int dp_ff_classify_device(dp_ctx_t *ctx, const dp_ff_input_t *dev_in, dp_ff_result_t *dev_out,
                          uint32_t n, void *stream);
/* The same for inputs and results in host memory (synchronous). */
int dp_ff_classify(dp_ctx_t *ctx, const dp_ff_input_t *in, dp_ff_result_t *out, uint32_t n);

/* The two tables alone over the reference's own key bytes -- what the
 * rte_acl classifiers behind lookup_batch are handed (AnyTable::lookup_batch,
 * tables.rs:313-326; MatchKey::as_key_into's fields back to back, big-endian,
 * match-action-derive/src/lib.rs:191-206):
 *   table DP_FF_REMOTE, RemoteKey<I>: proto 1, src_vni 4, dst_vni (GateVni, 0
 *     None) 4, destination 4 / 16, destination port 2 -- DP_FF_REMOTE_KEY_V4
 *     (15) or DP_FF_REMOTE_KEY_V6 (27) bytes;
 *   table DP_FF_LOCAL, LocalKey<I>: proto 1, src_vni 4, dst_vni 4, source 4 /
 *     16, source port 2, gate (SourceGate) 1 -- DP_FF_LOCAL_KEY_V4 (16) or
 *     DP_FF_LOCAL_KEY_V6 (28) bytes;
 * keys `stride` bytes apart (>= key_size), the key size naming the family.
 * dp_ff_key_from_match converts n of them to dp_ff_input_t (host code: no
 * device, no context; a remote key leaves the source zero, a local key the
 * destination); dp_ff_classify_match runs that table alone: per key
 * DP_FF_ROUTE with the matching rule's action (remote: dst_vni + dst_nat;
 * local: src_nat), else DP_FF_DESTINATION_MISS (remote) / DP_FF_SOURCE_MISS
 * (local).  DP_EINVAL: another table, key size, stride < key_size. */
enum dp_ff_table { DP_FF_REMOTE = 1, DP_FF_LOCAL = 2 };
#define DP_FF_REMOTE_KEY_V4 15u
#define DP_FF_REMOTE_KEY_V6 27u
#define DP_FF_LOCAL_KEY_V4 16u
#define DP_FF_LOCAL_KEY_V6 28u
int dp_ff_key_from_match(int table, const uint8_t *match, uint32_t key_size, uint32_t stride, uint32_t n,
                         dp_ff_input_t *out);
int dp_ff_classify_match(dp_ctx_t *ctx, int table, const uint8_t *match, uint32_t key_size,
                         uint32_t stride, uint32_t n, dp_ff_result_t *out);

/* ------------------------------------------------------------------------ */
/* Flow table: FlowTable                              */
/* (flow-entry/src/flow_table/table.rs:24-330) resident in HBM, consulted by */
/* the FlowLookup stage (nf_lookup.rs:34-55) and by the flow-aware branches  */
/* of IcmpErrorHandler (nat/src/icmp_handler/nf.rs:102-180), FlowFilter      */
/* (flow-filter/src/lib.rs:115-349) and AclFilter (acl-filter/src/lib.rs:    */
/* 62-138) for every context it is attached to.                              */
/*                                                                           */
/* The NAT state of the flow pairs the data path creates is carried:        */
/* port forwarding's (.port_fw_state) and masquerade's (.nat_state, with the */
/* allocation the SrcNat flow owns, released when that flow leaves the table:*/
/* a sweep, a remove, or a replacement -- at the end of the burst that       */
/* replaced it).  Every flow has a destination VPC.                          */
/*                                                                           */
/* Burst semantics are the reference pipeline's: FlowLookup, the flow-filter */
/* bypass decision and IcmpErrorHandler see flow states as they were when    */
/* the burst started; flows invalidated by the flow-filter (a miss, or an    */
/* outdated flow) are seen invalid by every AclFilter of the burst, and a    */
/* packet denied by the ACL invalidates its flows for the packets after it   */
/* (the pipeline runs FlowFilter over the whole burst, then the later stages */
/* packet by packet: flow-filter/src/lib.rs:352-363).                        */
/* ------------------------------------------------------------------------ */
typedef struct dp_flow_table dp_flow_table_t;

/* IpProtoKey variant (net/src/flows/flow_key.rs:360-365).  ICMP error keys
 * (IcmpProtoKey::ErrorMsgData) are never stored: no creator of flows makes
 * them, so dp_flow_insert rejects them and lookups of such keys miss. */
enum dp_flow_kind {
    DP_FLOW_TCP = 1,          /* sport / dport */
    DP_FLOW_UDP = 2,          /* sport / dport */
    DP_FLOW_ICMP_QUERY = 3,   /* IcmpProtoKey::QueryMsgData: sport = identifier, dport = 0 */
    DP_FLOW_ICMP_OTHER = 4    /* IcmpProtoKey::Unsupported: ports 0 */
};
/* FlowStatus (net/src/flows/flow_info.rs:37-49). */
enum dp_flow_status { DP_FLOW_ACTIVE = 0, DP_FLOW_CANCELLED = 1, DP_FLOW_EXPIRED = 2,
                      DP_FLOW_DETACHED = 3 };
/* FlowInfoFlags (flow_info.rs:142-149). */
enum dp_flow_flag { DP_FLOW_INITIATOR = 1u << 0, DP_FLOW_REQ_STATIC_NAT_SRC = 1u << 1,
                    DP_FLOW_REQ_STATIC_NAT_DST = 1u << 2 };

/* FlowKey (flow_key.rs:457-463): src_vpcd (0 = None), addresses of one
 * family (v4 in src[0..4] / dst[0..4], the rest zero), protocol key. */
typedef struct dp_flow_key {
    uint32_t src_vni;
    uint8_t family;           /* 4 or 6 */
    uint8_t kind;             /* enum dp_flow_kind */
    uint16_t pad;
    uint16_t sport, dport;
    uint8_t src[16];
    uint8_t dst[16];
} dp_flow_key_t;

/* A FlowInfo to insert (flow_info.rs:189-199). */
typedef struct dp_flow {
    dp_flow_key_t key;
    uint32_t dst_vni;         /* FlowInfoLocked.dst_vpcd (required, != 0) */
    uint32_t flags;           /* enum dp_flow_flag */
    uint32_t pad;
    int64_t genid;            /* FlowInfo.genid */
    uint64_t expires_at;      /* FlowInfo.expires_at, on the caller's clock */
} dp_flow_t;

/* A flow as stored.  `ref` names one stored FlowInfo (slot + fill tag); a
 * flow replaced or removed from the table no longer matches its ref. */
/* PortFwState.action (nat/src/common/mod.rs:14-19) */
enum dp_pf_action { DP_PF_NONE = 0, DP_PF_DST_NAT = 1, DP_PF_SRC_NAT = 2 };
/* NatFlowStatus (nat/src/common/mod.rs:34-45), shared by the two flows of a
 * port-forwarded pair */
enum dp_nat_flow_status { DP_NFS_ONE_WAY = 0, DP_NFS_TWO_WAY = 1, DP_NFS_ESTABLISHED = 2,
                          DP_NFS_RESET = 3, DP_NFS_C_CLOSING = 4, DP_NFS_S_CLOSING = 5,
                          DP_NFS_C_HALF_CLOSE = 6, DP_NFS_S_HALF_CLOSE = 7,
                          DP_NFS_LAST_ACK = 8, DP_NFS_CLOSED = 9 };
typedef struct dp_flow_info {
    uint64_t ref;             /* DP_FLOW_NONE: not found */
    uint32_t status;          /* enum dp_flow_status */
    uint32_t flags;
    uint32_t dst_vni;
    uint32_t pad;
    int64_t genid;
    uint64_t expires_at;
    uint64_t related;         /* ref of the related flow (FlowInfo.related), DP_FLOW_NONE */
    /* FlowInfoLocked.port_fw_state (nat/src/portfw/flow_state.rs:29-35) */
    uint8_t pf;               /* enum dp_pf_action (DP_PF_NONE: no state) */
    uint8_t pf_status;        /* enum dp_nat_flow_status */
    uint16_t pf_port;         /* use_port */
    uint32_t pf_rule;         /* id of the PortFwEntry its Weak names (dp_portfw_rule_t) */
    uint8_t pf_family;        /* use_ip family */
    uint8_t pad2[7];
    uint8_t pf_ip[16];        /* use_ip */
    /* FlowInfoLocked.nat_state (MasqueradeState, nat/src/masquerade/state.rs:
     * 13-20): action, with the status / use_ip / use_port in pf_status /
     * pf_ip / pf_port (pf_family) */
    uint8_t masq;             /* enum dp_pf_action (DP_PF_NONE: no state) */
    uint8_t masq_alloc;       /* 1: the state owns an allocation (the SrcNat flow) */
    uint16_t pad3;
    uint32_t idle_timeout_s;  /* MasqueradeState.idle_timeout */
} dp_flow_info_t;
#define DP_FLOW_NONE UINT64_MAX

/* dp_flow_insert per-flow results */
#define DP_FLOW_INSERTED 0
#define DP_FLOW_REPLACED 1    /* an existing flow of that key became Detached */
#define DP_EFLOWCAP (-28)     /* FlowTableError::CapacityExceeded (ENOSPC) */

/* `slots`: a power of two; the table holds at most slots / 2 flows.  The
 * capacity (FlowTable::set_capacity) defaults to FlowTable::DEFAULT_CAPACITY
 * (10M, table.rs:65) clamped to slots / 2. */
int dp_flow_table_create(int device_ordinal, uint64_t slots, dp_flow_table_t **out);
int dp_flow_table_destroy(dp_flow_table_t *ft);
int dp_flow_table_set_capacity(dp_flow_table_t *ft, uint64_t capacity);

/* FlowTable::insert for each flow in order (table.rs:134-260): the flow
 * becomes Active; an existing flow of the same key is Detached and replaced;
 * at capacity a new flow is refused (DP_EFLOWCAP).  `refs` / `results` may
 * be NULL.  Synchronous. */
int dp_flow_insert(dp_flow_table_t *ft, const dp_flow_t *flows, uint32_t n, uint64_t *refs,
                   int32_t *results);
/* FlowInfo::related_pair (flow_info.rs:290-339) then insert of both: exactly
 * one flow must have DP_FLOW_INITIATOR and the keys must differ.  The second
 * is admitted at capacity if the first is in the table and Active
 * (table.rs:221-233).  refs[2] / results[2] may be NULL. */
int dp_flow_insert_pair(dp_flow_table_t *ft, const dp_flow_t *a, const dp_flow_t *b,
                        uint64_t *refs, int32_t *results);
/* FlowTable::lookup (table.rs:267-275). */
int dp_flow_lookup(dp_flow_table_t *ft, const dp_flow_key_t *keys, uint32_t n,
                   dp_flow_info_t *out);
/* Current state of stored flows by ref (status etc.; ref DP_FLOW_NONE in
 * `out` when the ref no longer names a stored flow). */
int dp_flow_get(dp_flow_table_t *ft, const uint64_t *refs, uint32_t n, dp_flow_info_t *out);
/* FlowTable::remove (table.rs:282-295): the flow becomes Detached. */
int dp_flow_remove(dp_flow_table_t *ft, const dp_flow_key_t *keys, uint32_t n,
                   uint32_t *n_removed);
/* FlowInfo::invalidate_pair (flow_info.rs:435-455) / update_status. */
int dp_flow_invalidate(dp_flow_table_t *ft, const uint64_t *refs, uint32_t n);
int dp_flow_set_status(dp_flow_table_t *ft, uint64_t ref, uint32_t status);
/* The flow timers (FlowTable::start_timer, table.rs:160-213) up to `now`:
 * an Active flow with expires_at <= now becomes Expired and leaves the table;
 * a Cancelled or Expired flow leaves the table; a Detached one stays. */
int dp_flow_sweep(dp_flow_table_t *ft, uint64_t now, uint64_t *n_removed);
/* FlowTable::len / active_len (table.rs:297-317). */
int dp_flow_count(dp_flow_table_t *ft, uint64_t *len, uint64_t *active);
/* FlowLookup::new(name, Arc<FlowTable>) for this context's pipeline (and the
 * IcmpErrorHandler's table); NULL detaches (an empty flow table).  The table
 * must live on the context's device and outlive the attachment. */
int dp_ctx_attach_flow_table(dp_ctx_t *ctx, dp_flow_table_t *ft);


/* ------------------------------------------------------------------------ */
/* DPDK rx / tx burst glue: an rx burst of rte_mbufs  */
/* (RxQueue::receive, dpdk/src/queue/rx.rs:178-201) runs through the path in */
/* place in its mempool memory, and every delivered mbuf is left holding its */
/* serialized frame, ready for TxQueue::transmit (dpdk/src/queue/tx.rs:      */
/* 144-160).  The mempool region must be pinned and device-mapped            */
/* (hipHostRegister of the hugepage memzone): the kernel reads and rewrites  */
/* the frames over PCIe, no staging copies (the zero-copy host path).        */
/* Mbuf::raw_data (dpdk/src/mem.rs:502-522): the frame is the first segment, */
/* buf_addr + data_off, data_len bytes.                                      */
/* ------------------------------------------------------------------------ */

/* Byte offsets of the rte_mbuf fields this glue reads and writes; the
 * default is the rte_mbuf_core.h layout of the reference's DPDK (v26.03,
 * npins/sources.json: githedgehog/dpdk@fa7e361) on 64-bit targets. */
typedef struct dp_mbuf_layout {
    uint16_t buf_addr;    /* void *   */
    uint16_t data_off;    /* uint16_t */
    uint16_t nb_segs;     /* uint16_t */
    uint16_t port;        /* uint16_t */
    uint16_t pkt_len;     /* uint32_t */
    uint16_t data_len;    /* uint16_t */
    uint16_t buf_len;     /* uint16_t */
    uint16_t pad;
} dp_mbuf_layout_t;
#define DP_MBUF_LAYOUT_DPDK {0, 16, 20, 22, 36, 40, 54, 0}

/* Burst records for an rx burst: in[i].off = the frame's offset from
 * `pool_base`, .len = data_len, .iif = port_ifindex[port] (the driver's
 * PacketMeta.iif; `port_ifindex` NULL: the port number).  An mbuf whose frame
 * lies outside [pool_base, pool_base + pool_bytes), beyond 4 GiB of it, or
 * with less than DP_HEADROOM bytes of headroom, gets a record the pipeline
 * marks InternalFailure.  Host only (no device call). */
int dp_mbuf_burst_in(const void *pool_base, uint64_t pool_bytes, void *const *mbufs, uint32_t n,
                     const dp_mbuf_layout_t *layout, const uint32_t *port_ifindex,
                     uint32_t n_ports, dp_pkt_in_t *in);
/* Apply a burst's results to its mbufs: a Delivered mbuf's data_off,
 * data_len and pkt_len describe its serialized frame (prepend / trim of the
 * headroom, dpdk/src/mem.rs:547-590); other mbufs are left as received (the
 * caller frees them).  Host only. */
int dp_mbuf_burst_out(void *const *mbufs, uint32_t n, const dp_mbuf_layout_t *layout,
                      const dp_pkt_in_t *in, const dp_pkt_out_t *out);
/* dp_mbuf_burst_in, the pipeline over the mapped mempool region (zero copy),
 * dp_mbuf_burst_out.  `out` (host memory) receives every packet's result
 * (`meta`, may be NULL, the rest of its PacketMeta);
 * the caller transmits the Delivered mbufs on their out[i].oif and frees the
 * others.  Synchronous.  A pool that is not device-mapped fails with
 * DP_EINVAL (every out[i] InternalFailure). */
int dp_process_mbufs(dp_ctx_t *ctx, const void *pool_base, uint64_t pool_bytes,
                     void *const *mbufs, uint32_t n, const dp_mbuf_layout_t *layout,
                     const uint32_t *port_ifindex, uint32_t n_ports, dp_pkt_out_t *out,
                     dp_pkt_meta_t *meta, uint64_t *stats);

/* Introspection: bytes of the device table image and its parts (for
 * DESIGN.md / bench), and the last HIP error string. */
uint64_t dp_tables_device_bytes(const dp_ctx_t *ctx);
const char *dp_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* DPGPU_H */

/* SPDX-License-Identifier: Apache-2.0
 *
 * TEST INFRASTRUCTURE -- NOT PRODUCT CODE.
 *
 * CPU oracle: a plain C++ restatement of the reference (githedgehog/dataplane)
 * per-burst packet path, used only as the parity checker by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * (dataplane_amd/, libdpgpu.so) never links or calls it.
 *
 * Parity pinning: the reference is Rust and cannot be compiled here (no
 * cargo/rustc).  This restatement is pinned by the
 * reference's own known-answer tests transcribed into tests/golden/ (NAT
 * KATs of nat/src/static_nat/test.rs, ACL first-match of
 * acl/src/reference/table.rs, flow-filter priority, prefix masks, TTL chain,
 * VXLAN QoS preservation) -- see tests/test_oracle_kats.py.  Third-party
 * arithmetic (etherparse 0.21.0, prefix-trie 0.10.1, rapidhash 4.5.1) is
 * restated from their published behaviour; rapidhash-dependent values (ECMP
 * index, VXLAN UDP source port) are "parity unpinned" (SURVEY.md §8c).
 *
 * It exposes the same descriptor types as include/dpgpu.h so tests compare
 * the GPU path and the oracle on identical inputs.
 */
#ifndef DP_ORACLE_H
#define DP_ORACLE_H

#include "../include/dpgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dpo_tables dpo_tables_t;

/* Build oracle tables from the lowered descriptors (same semantics as
 * dp_tables_publish).  Returns 0 / negative errno. */
int dpo_tables_build(const dp_tables_desc_t *desc, dpo_tables_t **out);
/* The same as the next generation of `prev` (NULL: the first): the
 * port-forwarding entries are updated as PortFwTable::update does, so entry
 * ids carry over as dp_tables_publish carries them on one device. */
int dpo_tables_build2(const dp_tables_desc_t *desc, const dpo_tables_t *prev, dpo_tables_t **out);
/* Is port-forwarding entry `id` in these tables (its Weak upgrades)? */
int dpo_portfw_rule_alive(const dpo_tables_t *t, uint32_t id);
void dpo_tables_free(dpo_tables_t *t);

/* Run the reference stage sequence over a burst, in place, exactly like
 * dp_process_burst.  Single-threaded per call. */
int dpo_process_burst(const dpo_tables_t *t, uint8_t *buf, uint64_t buf_bytes,
                      const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta,
                      uint32_t n, uint64_t *stats);

/* Multi-threaded CPU baseline: splits the burst into bursts of `burst`
 * packets (DPDK PKT_BURST_SIZE = 64, dpdk/src/queue/rx.rs:174) over
 * `threads` threads.  Returns 0 / negative errno. */
int dpo_process_parallel(const dpo_tables_t *t, uint8_t *buf, uint64_t buf_bytes,
                         const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta,
                         uint32_t n, uint32_t burst, uint32_t threads);

/* Flow table (flow-entry/src/flow_table/table.rs) with the dp_flow_* semantics
 * of include/dpgpu.h; refs are indices of the FlowInfos the table made. */
typedef struct dpo_flows dpo_flows_t;
int dpo_flows_create(dpo_flows_t **out);
void dpo_flows_free(dpo_flows_t *fl);
int dpo_flows_set_capacity(dpo_flows_t *fl, uint64_t capacity);
int dpo_flow_insert(dpo_flows_t *fl, const dp_flow_t *flows, uint32_t n, uint64_t *refs,
                    int32_t *results);
int dpo_flow_insert_pair(dpo_flows_t *fl, const dp_flow_t *a, const dp_flow_t *b, uint64_t *refs,
                         int32_t *results);
int dpo_flow_lookup(dpo_flows_t *fl, const dp_flow_key_t *keys, uint32_t n, dp_flow_info_t *out);
int dpo_flow_get(dpo_flows_t *fl, const uint64_t *refs, uint32_t n, dp_flow_info_t *out);
int dpo_flow_remove(dpo_flows_t *fl, const dp_flow_key_t *keys, uint32_t n, uint32_t *n_removed);
int dpo_flow_invalidate(dpo_flows_t *fl, const uint64_t *refs, uint32_t n);
int dpo_flow_set_status(dpo_flows_t *fl, uint64_t ref, uint32_t status);
int dpo_flow_sweep(dpo_flows_t *fl, uint64_t now, uint64_t *n_removed);
int dpo_flow_count(dpo_flows_t *fl, uint64_t *len, uint64_t *active);
/* NatAllocatorWriter::update_nat_allocator for the tables `t` (what
 * dp_tables_publish does for every flow table attached on the device): keep
 * the allocator of an unchanged masquerade configuration, drop it (and
 * invalidate the masquerade flows) for one without masquerade, else build a
 * new one and carry the flows it can still serve.  A burst runs it too. */
int dpo_flows_sync(dpo_flows_t *fl, const dpo_tables_t *t);
/* Instant::now() for the bursts that follow (DP_OPT_CLOCK, nanoseconds). */
int dpo_flows_set_clock(dpo_flows_t *fl, uint64_t now);
/* One burst through the pipeline with FlowLookup on `fl` (NULL: an empty
 * flow table), in the reference's burst order; meta[i].flow_ref is each
 * packet's PacketMeta.flow_info (DP_FLOW_NONE: none). */
int dpo_process_burst_flows(const dpo_tables_t *t, dpo_flows_t *fl, uint8_t *buf,
                            uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                            dp_pkt_meta_t *meta, uint32_t n, uint64_t *stats);

/* Primitive restatements exposed for unit tests. */
uint16_t dpo_checksum_ipv4_header(const uint8_t *hdr, uint32_t hlen);
/* LPM of one address in one FIB: returns route nh index or -1. */
int64_t dpo_lpm(const dpo_tables_t *t, uint32_t fib, uint8_t family,
                const uint8_t *addr);
/* First-match ACL over a table: returns rule index or -1. */
int64_t dpo_acl_lookup(const dpo_tables_t *t, uint8_t family, uint8_t proto,
                       uint32_t src_vni, uint32_t dst_vni, const uint8_t *src,
                       const uint8_t *dst, int has_ports, uint16_t sport,
                       uint16_t dport);
/* AclFilter's decision for each key (dpgpu.h dp_acl_classify). */
int dpo_acl_classify(const dpo_tables_t *t, const dp_acl_key_t *keys, dp_acl_result_t *out, uint32_t n);
// FlowFilterContext::lookup_batch (dpgpu.h dp_ff_classify); stage 0 both
// tables, 1 the remote rules alone, 2 the local rules alone
int dpo_ff_classify(const dpo_tables_t *t, const dp_ff_input_t *in, dp_ff_result_t *out, uint32_t n, int stage);
/* Static NAT find_{src,dst}_mapping: returns 1 if mapped (new addr/port
 * written, port 0 = unchanged), 0 if not. kind: 0 dst, 1 src. */
int dpo_nat_lookup(const dpo_tables_t *t, uint32_t kind, uint32_t src_vni,
                   uint32_t dst_vni, const uint8_t *addr4, int has_port,
                   uint16_t port, uint8_t *new_addr4, uint16_t *new_port);
/* rapidhash-style 64-bit hash restatement (parity unpinned). */
uint64_t dpo_hash_bytes(const uint8_t *p, uint32_t len);
/* Packet::new + Packet::serialize of one frame (tx of a packet rebuilt from
 * an output frame); returns the transmitted length or -1. */
int dpo_reserialize(const uint8_t *frame, uint32_t len, uint8_t *out, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif

// SPDX-License-Identifier: Apache-2.0
//
// Seeded synthetic workloads for the five BASELINE.json configurations
// (SURVEY.md §8d).  Produces lowered tables (dp_tables_desc_t) and a burst
// buffer (frames with DP_HEADROOM in front, 16-byte aligned) with valid
// checksums.  Harness code: used by bench.py and the tests, never by the
// packet path itself.
//
//   C1  64B IPv4/UDP underlay, 1k-route LPM (CPU loopback config)
//   C2  64B IPv4/UDP overlay (seeded decap), 1M routes + 10k ACL + static NAT
//   C3  IMIX 7:4:1 of 60/566/1514 B, C2 tables
//   C4  VXLAN-in-IPv4 (110 B): real decap + LPM + NAT + re-encap
//   C5  80/20 IPv4/IPv6, 1M v4 + 200k v6 routes, 10k+10k ACL, NAT44
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/dpgpu.h"

namespace {

struct Rng {  // splitmix64 seeded xoshiro256**
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (int i = 0; i < 4; i++) {
      seed += 0x9E3779B97F4A7C15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      s[i] = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  uint32_t u32() { return (uint32_t)(next() >> 32); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

inline void put16(uint8_t *p, uint16_t v) { p[0] = v >> 8; p[1] = v & 0xff; }
inline void put32(uint8_t *p, uint32_t v) { p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v; }

uint16_t csum_fold(uint64_t s) {
  while (s >> 16) s = (s & 0xffff) + (s >> 16);
  return (uint16_t)~s;
}
uint64_t sum_bytes(const uint8_t *p, size_t n) {
  uint64_t s = 0;
  size_t i = 0;
  for (; i + 1 < n; i += 2) s += (uint32_t)((p[i] << 8) | p[i + 1]);
  if (i < n) s += (uint32_t)(p[i] << 8);
  return s;
}

dp_prefix_t pfx4(uint32_t a, int len) {
  dp_prefix_t p{};
  p.family = 4;
  p.len = (uint8_t)len;
  uint32_t m = len == 0 ? 0 : (0xffffffffu << (32 - len));
  put32(p.addr, a & m);
  return p;
}
dp_prefix_t pfx6(const uint8_t *a, int len) {
  dp_prefix_t p{};
  p.family = 6;
  p.len = (uint8_t)len;
  for (int i = 0; i < 16; i++) {
    int bits = std::max(0, std::min(8, len - 8 * i));
    p.addr[i] = bits == 0 ? 0 : (uint8_t)(a[i] & (0xff << (8 - bits)));
  }
  return p;
}
dp_ipaddr_t ip4(uint32_t a) { dp_ipaddr_t r{}; r.family = 4; put32(r.addr, a); return r; }

}  // namespace

extern "C" {

typedef struct dpw_config {
  uint32_t config;        // 1..5
  uint32_t n_packets;
  uint64_t seed;
  uint32_t n_routes_v4;   // 0 = config default
  uint32_t n_routes_v6;
  uint32_t n_acl;         // per family; 0 = config default (C1: none)
  uint32_t n_nat;         // /24 maps per direction
  uint32_t n_vni;         // source VPCs
  uint32_t tcp_percent;   // share of TCP among L4 (default 0: UDP only)
  uint32_t layout;        // 0: packed (DP_HEADROOM in front, 16-byte aligned slots);
                          // 1: DPDK mbuf (RTE_PKTMBUF_HEADROOM = 128 in front of a
                          //    64-byte aligned data start, slots 64-byte aligned)
} dpw_config_t;

struct dpw_workload {
  std::vector<dp_fib_t> fibs;
  std::vector<dp_vni_fib_t> vnis;
  std::vector<dp_route_t> routes;
  std::vector<dp_route_nh_t> nhs;
  std::vector<dp_fib_entry_t> entries;
  std::vector<dp_instr_t> instrs;
  std::vector<dp_iface_t> ifaces;
  std::vector<dp_adjacency_t> adjs;
  std::vector<dp_rule_t> acl4, acl6, ffr4, ffl4, ffr6, ffl6;
  std::vector<dp_acl_default_t> acl_def;
  std::vector<dp_nat_table_t> nat_tabs;
  std::vector<dp_nat_entry_t> nat_ents;
  std::vector<dp_port_range_t> nat_prs;
  std::vector<dp_nat_range_t> nat_ranges;
  dp_tables_desc_t desc{};
  std::vector<uint8_t> buf;
  std::vector<dp_pkt_in_t> in;
  uint64_t payload_bytes = 0;
};
typedef struct dpw_workload dpw_workload_t;

}  // extern "C"

namespace {

const uint8_t kIfMac[6] = {0x02, 0x00, 0x00, 0x00, 0x00, 0x01};
const uint8_t kPeerMac[6] = {0x02, 0x00, 0x00, 0x00, 0xee, 0x01};

dp_rule_t wildcard_rule(int fam) {
  dp_rule_t r{};
  r.family = (uint8_t)fam;
  r.src.family = r.dst.family = (uint8_t)fam;
  r.sport_lo = 0; r.sport_hi = 65535; r.dport_lo = 0; r.dport_hi = 65535;
  return r;
}

int rand_len_v4(Rng &r) {  // BGP-like histogram, ~55% /24
  double u = r.unit();
  if (u < 0.001) return 8;
  if (u < 0.02) return 9 + (int)r.below(7);
  if (u < 0.07) return 16;
  if (u < 0.37) return 17 + (int)r.below(7);
  if (u < 0.92) return 24;
  return 25 + (int)r.below(8);
}
int rand_len_v6(Rng &r) {  // /16-/64 histogram, ~50% /48
  double u = r.unit();
  if (u < 0.05) return 16 + (int)r.below(16);
  if (u < 0.35) return 32 + (int)r.below(16);
  if (u < 0.85) return 48;
  return 49 + (int)r.below(16);
}

struct Builder {
  dpw_workload &w;
  Rng rng;
  int cfg;
  uint32_t n_vni;
  Builder(dpw_workload &w_, uint64_t seed, int c) : w(w_), rng(seed), cfg(c), n_vni(4) {}

  uint32_t add_entry(const std::vector<dp_instr_t> &ins) {
    dp_fib_entry_t e{(uint32_t)w.instrs.size(), (uint32_t)ins.size()};
    w.instrs.insert(w.instrs.end(), ins.begin(), ins.end());
    w.entries.push_back(e);
    w.nhs.push_back(dp_route_nh_t{(uint32_t)w.entries.size() - 1, 1});
    return (uint32_t)w.nhs.size() - 1;
  }
};

}  // namespace

extern "C" {

void dpw_free(dpw_workload_t *w) { delete w; }

// Build tables + burst.  Returns 0 or a negative errno.
int dpw_build(const dpw_config_t *c, dpw_workload_t **out) {
  if (!c || !out || c->config < 1 || c->config > 5) return DP_EINVAL;
  auto W = std::make_unique<dpw_workload>();
  dpw_workload &w = *W;
  Builder B(w, c->seed ? c->seed : 0x5eed, (int)c->config);
  Rng &R = B.rng;
  const int cfg = (int)c->config;
  const bool overlay = cfg != 1;
  const bool vxlan = cfg == 4;
  const bool v6mix = cfg == 5;
  uint32_t n_v4 = c->n_routes_v4 ? c->n_routes_v4 : (cfg == 1 ? 1000 : 1000000);
  uint32_t n_v6 = c->n_routes_v6 ? c->n_routes_v6 : (v6mix ? 200000 : 0);
  uint32_t n_acl = overlay ? (c->n_acl ? c->n_acl : 10000) : 0;
  uint32_t n_nat = overlay ? (c->n_nat ? c->n_nat : 256) : 0;
  uint32_t n_vni = c->n_vni ? c->n_vni : 4;
  const uint32_t kDstVni = 2000;

  // ---------------- interfaces: iif 1 (underlay / VRF 0), oifs 10..13
  {
    dp_iface_t i{};
    i.ifindex = 1; i.admin_state = DP_IF_UP; i.oper_state = DP_IF_UP;
    i.iftype = DP_IFT_ETHERNET; i.attach = DP_ATTACH_VRF; i.vrf_id = 0;
    memcpy(i.mac, kIfMac, 6);
    w.ifaces.push_back(i);
    for (int k = 0; k < 4; k++) {
      dp_iface_t o = i;
      o.ifindex = 10 + k;
      o.mac[5] = (uint8_t)(0x10 + k);
      w.ifaces.push_back(o);
    }
  }
  // ---------------- FIBs: 0 underlay (vrf 0), 1..n_vni source VPCs, last = dst VPC
  {
    dp_fib_t u{};
    u.vrf_id = 0;
    u.flags = DP_FIB_VTEP_HAS_IP | DP_FIB_VTEP_HAS_MAC;
    u.vtep_ip = ip4(0x64400001);  // 100.64.0.1
    memcpy(u.vtep_mac, kIfMac, 6);
    w.fibs.push_back(u);
    for (uint32_t k = 0; k < n_vni; k++) {
      dp_fib_t f = u;
      f.vrf_id = 100 + k;
      w.fibs.push_back(f);
      w.vnis.push_back(dp_vni_fib_t{1000 + k, 1 + k});
    }
    dp_fib_t d = u;
    d.vrf_id = 200;
    w.fibs.push_back(d);
    w.vnis.push_back(dp_vni_fib_t{kDstVni, 1 + n_vni});
  }
  const uint32_t fib_under = 0, fib_dst = 1 + n_vni;
  // ---------------- next hops: 64 on 4 oifs, adjacencies resolved
  std::vector<uint32_t> nh_egress, nh_encap;
  for (int j = 0; j < 64; j++) {
    uint32_t nhip = 0xc0000200u + (uint32_t)j + 1;  // 192.0.2.x
    uint32_t oif = 10 + (j & 3);
    dp_adjacency_t a{};
    a.addr = ip4(nhip);
    a.ifindex = oif;
    uint8_t mac[6] = {0x02, 0x00, 0x00, 0x00, 0x77, (uint8_t)(j + 1)};
    memcpy(a.mac, mac, 6);
    w.adjs.push_back(a);
    dp_instr_t eg{};
    eg.kind = DP_INSTR_EGRESS;
    eg.flags = DP_INSTR_HAS_IFINDEX | DP_INSTR_HAS_ADDR;
    eg.ifindex = oif;
    eg.addr = ip4(nhip);
    nh_egress.push_back(B.add_entry({eg}));
    if (vxlan) {
      dp_instr_t en{};
      en.kind = DP_INSTR_ENCAP_VXLAN;
      en.flags = DP_INSTR_HAS_DMAC;
      en.vni = kDstVni;
      en.addr = ip4(0x64410000u + (uint32_t)j + 1);  // remote VTEP 100.65.0.x
      uint8_t rm[6] = {0x02, 0x00, 0x00, 0x00, 0x88, (uint8_t)(j + 1)};
      memcpy(en.mac, rm, 6);
      nh_encap.push_back(B.add_entry({en, eg}));
    }
  }
  // local VTEP route in the underlay (decap)
  uint32_t nh_local = 0;
  {
    dp_instr_t lo{};
    lo.kind = DP_INSTR_LOCAL;
    lo.ifindex = 1;
    nh_local = B.add_entry({lo});
  }
  const std::vector<uint32_t> &route_nhs = vxlan ? nh_encap : nh_egress;
  const uint32_t route_fib = overlay ? fib_dst : fib_under;
  // ---------------- v4 routes (+ an explicit default so misses are forwarded)
  std::vector<dp_route_t> v4r;
  w.routes.reserve(n_v4 + n_v6 + 8);
  for (uint32_t k = 0; k < n_v4; k++) {
    int len = rand_len_v4(R);
    uint32_t a = (cfg == 1) ? R.u32() : (0x0a000000u | (R.u32() & 0x00ffffffu));  // overlay in 10/8
    if (cfg != 1 && len < 8) len = 8;
    dp_route_t r{};
    r.prefix = pfx4(a, len);
    r.fib = route_fib;
    r.nh = route_nhs[R.below((uint32_t)route_nhs.size())];
    w.routes.push_back(r);
  }
  {
    dp_route_t d{};
    d.prefix = pfx4(0, 0);
    d.fib = route_fib;
    d.nh = route_nhs[0];
    w.routes.push_back(d);
  }
  if (vxlan) {
    dp_route_t l{};
    l.prefix = pfx4(0x64400001u, 32);
    l.fib = fib_under;
    l.nh = nh_local;
    w.routes.push_back(l);
  }
  // ---------------- v6 routes (C5), egress via v4 next hops is fine: Egress
  // resolves the adjacency of the instruction's next-hop address.
  std::vector<std::array<uint8_t, 17>> v6pfx;
  for (uint32_t k = 0; k < n_v6; k++) {
    uint8_t a[16] = {0x20, 0x01, 0x0d, 0xb8};
    for (int i = 4; i < 16; i++) a[i] = (uint8_t)R.u32();
    int len = rand_len_v6(R);
    if (len < 32) len = 32;
    dp_route_t r{};
    r.prefix = pfx6(a, len);
    r.fib = route_fib;
    r.nh = route_nhs[R.below((uint32_t)route_nhs.size())];
    w.routes.push_back(r);
    std::array<uint8_t, 17> x;
    memcpy(x.data(), r.prefix.addr, 16);
    x[16] = (uint8_t)len;
    v6pfx.push_back(x);
  }
  if (n_v6) {
    dp_route_t d{};
    d.prefix.family = 6;
    d.prefix.len = 0;
    d.fib = route_fib;
    d.nh = route_nhs[0];
    w.routes.push_back(d);
  }

  // ---------------- overlay tables: flow filter, ACL, NAT
  // src VPC k (VNI 1000+k) peers with the dst VPC (VNI 2000).
  // private space of VPC k: 10.(16k..16k+15).0.0/12-ish; NAT publics 172.16/12
  std::vector<uint32_t> src_nat_priv, src_nat_pub, dst_nat_pub, dst_nat_priv;
  // every 4th source-NAT map is PAT (ports kPatPortLo..65535)
  const uint16_t kPatPortLo = 1024;
  auto is_pat = [](uint32_t k) { return (k & 3) == 3; };
  // per v4 ACL rule: the NAT /24 its src / dst prefix was built over (0: none)
  std::vector<std::array<uint32_t, 2>> acl_anchor;
  if (overlay) {
    for (uint32_t k = 0; k < n_nat; k++) {
      src_nat_priv.push_back(0x0a000000u | ((k % 240u) << 16) | ((k / 240u) << 8));   // 10.x.y.0/24
      src_nat_pub.push_back(0xac100000u | (k << 8));                                   // 172.16.k.0/24
      dst_nat_pub.push_back(0xac200000u | (k << 8));                                   // 172.32.k.0/24
      dst_nat_priv.push_back(0x0a800000u | (k << 8));                                  // 10.128.k.0/24
    }
    for (uint32_t s = 0; s < n_vni; s++) {
      uint32_t svni = 1000 + s;
      // remote (stage 1): peer public /24s with static dst NAT, plus default
      for (uint32_t k = 0; k < n_nat; k++) {
        dp_rule_t r = wildcard_rule(4);
        r.proto_mask = 0;
        r.vni_a = svni;
        r.dst = pfx4(dst_nat_pub[k], 24);
        r.priority = ((24 + 1) << 1);
        r.action = kDstVni;
        r.action2 = DP_NAT_STATIC;
        w.ffr4.push_back(r);
      }
      // the peer's routed space 10/8 (not a wildcard: other destinations miss
      // the remote stage and are Filtered)
      dp_rule_t d = wildcard_rule(4);
      d.vni_a = svni; d.dst = pfx4(0x0a000000u, 8); d.priority = (8 + 1) << 1;
      d.action = kDstVni; d.action2 = DP_NAT_NONE;
      w.ffr4.push_back(d);
      dp_rule_t d6 = wildcard_rule(6);
      d6.vni_a = svni; d6.priority = (0 + 1) << 1; d6.action = kDstVni; d6.action2 = DP_NAT_NONE;
      w.ffr6.push_back(d6);
      // local (stage 2): own private /24s with static src NAT, plus default
      for (uint32_t k = s; k < n_nat; k += n_vni) {
        dp_rule_t r = wildcard_rule(4);
        r.vni_a = svni; r.vni_b = kDstVni;
        r.src = pfx4(src_nat_priv[k], 24);
        if (is_pat(k)) { r.sport_lo = kPatPortLo; r.sport_hi = 65535; }
        r.priority = ((24 + 1) << 1);
        r.action = DP_NAT_STATIC;
        w.ffl4.push_back(r);
      }
      // own routed space 10/8 (sources outside it miss the local stage)
      dp_rule_t l = wildcard_rule(4);
      l.vni_a = svni; l.vni_b = kDstVni; l.src = pfx4(0x0a000000u, 8); l.priority = (8 + 1) << 1;
      l.action = DP_NAT_NONE;
      w.ffl4.push_back(l);
      dp_rule_t l6 = wildcard_rule(6);
      l6.vni_a = svni; l6.vni_b = kDstVni; l6.priority = 2; l6.action = DP_NAT_NONE;
      w.ffl6.push_back(l6);
      // NAT tables of src VPC s: src_nat[(s, dst)] and dst_nat[s]
      dp_nat_table_t st{DP_NAT_TABLE_SRC, svni, kDstVni, (uint32_t)w.nat_ents.size(), 0};
      for (uint32_t k = s; k < n_nat; k += n_vni) {
        dp_nat_entry_t e{};
        e.prefix = pfx4(src_nat_priv[k], 24);
        e.first_range = (uint32_t)w.nat_ranges.size();
        e.n_ranges = 1;
        dp_nat_range_t rg{};
        put32(rg.orig_lo_ip, src_nat_priv[k]); put32(rg.orig_hi_ip, src_nat_priv[k] | 0xff);
        rg.orig_hi_port = 65535;
        put32(rg.tgt_lo_ip, src_nat_pub[k]); put32(rg.tgt_hi_ip, src_nat_pub[k] | 0xff);
        rg.tgt_hi_port = 65535;
        if (is_pat(k)) {
          // PAT (NatTableValue::Pat): 256 addresses x ports 1024..65535 onto
          // 252 addresses x ports 0..65535 -- equal sizes (256 * 64512 =
          // 252 * 65536), one range, offset 0; a mapped port 0 is rejected
          e.is_pat = 1;
          e.first_port_range = (uint32_t)w.nat_prs.size();
          e.n_port_ranges = 1;
          w.nat_prs.push_back(dp_port_range_t{kPatPortLo, 65535});
          e.size = 256ull * (65536 - kPatPortLo);
          rg.orig_lo_port = kPatPortLo;
          put32(rg.tgt_hi_ip, src_nat_pub[k] + 251);
          rg.tgt_lo_port = 0;
        } else {
          e.size = 256;
        }
        w.nat_ranges.push_back(rg);
        w.nat_ents.push_back(e);
        st.n_entries++;
      }
      w.nat_tabs.push_back(st);
      dp_nat_table_t dt{DP_NAT_TABLE_DST, svni, 0, (uint32_t)w.nat_ents.size(), 0};
      for (uint32_t k = 0; k < n_nat; k++) {
        dp_nat_entry_t e{};
        e.prefix = pfx4(dst_nat_pub[k], 24);
        e.first_range = (uint32_t)w.nat_ranges.size();
        e.n_ranges = 1;
        e.size = 256;
        dp_nat_range_t rg{};
        put32(rg.orig_lo_ip, dst_nat_pub[k]); put32(rg.orig_hi_ip, dst_nat_pub[k] | 0xff);
        rg.orig_hi_port = 65535;
        put32(rg.tgt_lo_ip, dst_nat_priv[k]); put32(rg.tgt_hi_ip, dst_nat_priv[k] | 0xff);
        rg.tgt_hi_port = 65535;
        w.nat_ranges.push_back(rg);
        w.nat_ents.push_back(e);
        dt.n_entries++;
      }
      w.nat_tabs.push_back(dt);
      // ACL: n_acl rules per family spread over the source VPCs, default allow
      w.acl_def.push_back(dp_acl_default_t{svni, kDstVni, DP_ACL_ALLOW});
    }
    for (int fam = 4; fam <= (v6mix ? 6 : 4); fam += 2) {
      for (uint32_t k = 0; k < n_acl; k++) {
        dp_rule_t r = wildcard_rule(fam);
        uint32_t s = k % n_vni;
        r.vni_a = 1000 + s;
        r.vni_b = kDstVni;
        uint32_t pr = R.below(3);
        if (pr == 0) { r.proto_val = 17; r.proto_mask = 0xff; }
        else if (pr == 1) { r.proto_val = 6; r.proto_mask = 0xff; }
        int sl, dl;
        if (fam == 4) {
          sl = 16 + (int)R.below(13); dl = 16 + (int)R.below(13);
          uint32_t sa = 0x0a000000u | (R.u32() & 0x00ffffffu), da = 0x0a000000u | (R.u32() & 0x00ffffffu);
          uint32_t sanc = 0, danc = 0;
          // half of the rules sit over one of the VPC's source-NAT /24s and
          // half over a destination-NAT public /24 (anchored: a packet steered
          // to the rule keeps an address inside that /24, so steering toward
          // ACL rules keeps the NAT share)
          if (n_nat && R.below(2) == 0) {
            uint32_t kk = s + n_vni * R.below(std::max<uint32_t>(1, (n_nat - s + n_vni - 1) / n_vni));
            if (kk >= n_nat) kk = s;
            sanc = src_nat_priv[kk];
            sl = 20 + (int)R.below(9);
            sa = sanc | (R.u32() & 0xff);
          }
          if (n_nat && R.below(2) == 0) {
            danc = dst_nat_pub[R.below(n_nat)];
            dl = 22 + (int)R.below(7);
            da = danc | (R.u32() & 0xff);
          }
          r.src = pfx4(sa, sl);
          r.dst = pfx4(da, dl);
          acl_anchor.push_back({sanc, danc});
        } else {
          uint8_t a[16] = {0x20, 0x01, 0x0d, 0xb8}, b[16] = {0x20, 0x01, 0x0d, 0xb8};
          for (int i = 4; i < 16; i++) { a[i] = (uint8_t)R.u32(); b[i] = (uint8_t)R.u32(); }
          r.src = pfx6(a, 40 + (int)R.below(40));
          r.dst = pfx6(b, 40 + (int)R.below(40));
        }
        uint32_t pk = R.below(3);
        if (pk == 1) { r.dport_lo = r.dport_hi = (uint16_t)(1024 + R.below(64000)); }
        else if (pk == 2) { r.dport_lo = (uint16_t)(1024 + R.below(32000)); r.dport_hi = (uint16_t)(r.dport_lo + R.below(20000)); }
        r.action = R.below(10) == 0 ? DP_ACL_DENY : DP_ACL_ALLOW;
        (fam == 4 ? w.acl4 : w.acl6).push_back(r);
      }
    }
  }

  // ---------------- packets
  uint32_t n = c->n_packets;
  w.in.resize(n);
  // frame sizes
  std::vector<uint16_t> flen(n);
  for (uint32_t i = 0; i < n; i++) {
    uint16_t L = 60;
    if (cfg == 3) { uint32_t u = R.below(12); L = u < 7 ? 60 : (u < 11 ? 566 : 1514); }
    if (v6mix && R.below(5) == 0) L = 80;  // v6 marker (14+40+8+18)
    if (vxlan) L = 110;
    flen[i] = L;
  }
  uint64_t off = 0;
  std::vector<uint32_t> offs(n);
  const uint64_t hr = c->layout == 1 ? 128 : DP_HEADROOM, al = c->layout == 1 ? 64 : 16;
  for (uint32_t i = 0; i < n; i++) {
    off += hr;
    offs[i] = (uint32_t)off;
    off += flen[i];
    off = (off + al - 1) & ~(al - 1);  // next slot aligned
  }
  w.buf.assign(off + 64, 0);
  std::vector<uint32_t> acl_hit_pool;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t *f = w.buf.data() + offs[i];
    uint16_t L = flen[i];
    bool is6 = v6mix && L == 80;
    uint32_t s = R.below(n_vni);
    uint32_t svni = 1000 + s;
    bool tcp = c->tcp_percent && R.below(100) < c->tcp_percent;
    int o = 0;
    if (vxlan) {
      // outer Eth / IPv4 / UDP 4789 / VXLAN(svni)
      memcpy(f, kIfMac, 6); memcpy(f + 6, kPeerMac, 6); put16(f + 12, 0x0800);
      uint8_t *ip = f + 14;
      uint16_t tot = (uint16_t)(L - 14);
      ip[0] = 0x45; ip[1] = (uint8_t)(R.below(64) << 2); put16(ip + 2, tot); put16(ip + 4, (uint16_t)R.u32());
      ip[6] = 0x40; ip[7] = 0; ip[8] = 64; ip[9] = 17;
      put32(ip + 12, 0x64410000u + 1 + R.below(64)); put32(ip + 16, 0x64400001u);
      put16(ip + 10, 0); put16(ip + 10, csum_fold(sum_bytes(ip, 20)));
      uint8_t *u = ip + 20;
      put16(u, (uint16_t)(49152 + R.below(16384))); put16(u + 2, 4789); put16(u + 4, (uint16_t)(tot - 20)); put16(u + 6, 0);
      uint8_t *vx = u + 8;
      vx[0] = 0x08; vx[1] = vx[2] = vx[3] = 0; vx[4] = (uint8_t)(svni >> 16); vx[5] = (uint8_t)(svni >> 8); vx[6] = (uint8_t)svni; vx[7] = 0;
      o = 50;
    }
    uint8_t *e = f + o;
    uint16_t il = (uint16_t)(L - o);
    memcpy(e, kIfMac, 6); memcpy(e + 6, kPeerMac, 6);
    if (vxlan) { e[0] = 0x02; e[5] = 0x99; }  // inner MACs are ignored by the gateway
    put16(e + 12, is6 ? 0x86dd : 0x0800);
    uint8_t *ip = e + 14;
    uint8_t *l4;
    uint16_t l4len;
    uint32_t sip = 0, dip = 0;
    int steer_dp = -1;  // destination port inside the steered ACL rule's range
    uint8_t s6[16], d6[16];
    if (!is6) {
      if (overlay) {
        // src: half from this VPC's NATed private /24s
        if (R.below(2) == 0 && n_nat) {
          uint32_t k = s + n_vni * R.below(std::max<uint32_t>(1, (n_nat - s + n_vni - 1) / n_vni));
          if (k >= n_nat) k = s;
          sip = src_nat_priv[k] | (1 + R.below(254));
        } else {
          sip = 0x0a000000u | (R.u32() & 0x00ffffffu);
        }
        // dst: half toward NATed public /24s, else a routed 10/8 address
        if (R.below(2) == 0 && n_nat) dip = dst_nat_pub[R.below(n_nat)] | (1 + R.below(254));
        else {
          const dp_route_t &rr = w.routes[R.below(n_v4)];
          uint32_t net = (uint32_t)rr.prefix.addr[0] << 24 | (uint32_t)rr.prefix.addr[1] << 16 | (uint32_t)rr.prefix.addr[2] << 8 | rr.prefix.addr[3];
          uint32_t span = rr.prefix.len >= 32 ? 0 : (0xffffffffu >> rr.prefix.len);
          dip = net | (R.u32() & span);
        }
        // ACL: 80% of packets are steered toward a random rule of their pair
        if (n_acl && R.below(5) != 0) {
          uint32_t rk = s + n_vni * R.below(std::max<uint32_t>(1, n_acl / n_vni));
          if (rk < w.acl4.size()) {
            const dp_rule_t &ar = w.acl4[rk];
            uint32_t sn = (uint32_t)ar.src.addr[0] << 24 | (uint32_t)ar.src.addr[1] << 16 | (uint32_t)ar.src.addr[2] << 8 | ar.src.addr[3];
            uint32_t dn = (uint32_t)ar.dst.addr[0] << 24 | (uint32_t)ar.dst.addr[1] << 16 | (uint32_t)ar.dst.addr[2] << 8 | ar.dst.addr[3];
            sip = sn | (R.u32() & (ar.src.len >= 32 ? 0 : (0xffffffffu >> ar.src.len)));
            dip = dn | (R.u32() & (ar.dst.len >= 32 ? 0 : (0xffffffffu >> ar.dst.len)));
            // anchored prefixes: stay inside the NAT /24 (which holds the prefix
            // when it is longer than /24, else is inside it)
            const uint32_t sanc = acl_anchor[rk][0], danc = acl_anchor[rk][1];
            if (sanc && ar.src.len <= 24) sip = sanc | (1 + R.below(254));
            if (danc && ar.dst.len <= 24) dip = danc | (1 + R.below(254));
            if (ar.proto_mask) tcp = ar.proto_val == 6;
            steer_dp = (int)ar.dport_lo + (int)R.below((uint32_t)ar.dport_hi - ar.dport_lo + 1);
            if (steer_dp < 1024) steer_dp = -1;  // wildcard: keep the random port
          }
        }
        // flow-filter misses: 3% toward a destination no peering exposes
        // (remote stage miss), 2% from a source outside the VPC's space
        // (local stage miss) -- both Filtered
        const uint32_t u = R.below(100);
        if (u < 3) dip = 0xc0a80000u | (R.u32() & 0xffffu);        // 192.168/16
        else if (u < 5) sip = 0x647f0000u | (R.u32() & 0xffffu);   // 100.127/16
      } else {
        sip = 0x0a000000u | (R.u32() & 0x00ffffffu);
        const dp_route_t &rr = w.routes[R.below(n_v4)];
        uint32_t net = (uint32_t)rr.prefix.addr[0] << 24 | (uint32_t)rr.prefix.addr[1] << 16 | (uint32_t)rr.prefix.addr[2] << 8 | rr.prefix.addr[3];
        uint32_t span = rr.prefix.len >= 32 ? 0 : (0xffffffffu >> rr.prefix.len);
        dip = net | (R.u32() & span);
      }
      if ((sip >> 28) == 0xe) sip &= 0x0fffffff;
      l4 = ip + 20;
      l4len = (uint16_t)(il - 34);
      ip[0] = 0x45; ip[1] = 0; put16(ip + 2, (uint16_t)(il - 14)); put16(ip + 4, (uint16_t)R.u32());
      ip[6] = 0x40; ip[7] = 0; ip[8] = 64; ip[9] = tcp ? 6 : 17;
      put32(ip + 12, sip); put32(ip + 16, dip);
      put16(ip + 10, 0); put16(ip + 10, csum_fold(sum_bytes(ip, 20)));
    } else {
      s6[0] = 0x20; s6[1] = 0x01; s6[2] = 0x0d; s6[3] = 0xb8;
      for (int k = 4; k < 16; k++) s6[k] = (uint8_t)R.u32();
      const auto &pp = v6pfx[R.below((uint32_t)v6pfx.size())];
      memcpy(d6, pp.data(), 16);
      for (int k = pp[16] / 8 + 1; k < 16; k++) d6[k] = (uint8_t)R.u32();
      l4 = ip + 40;
      l4len = (uint16_t)(il - 54);
      ip[0] = 0x60; ip[1] = 0; ip[2] = 0; ip[3] = 0;
      put16(ip + 4, l4len); ip[6] = tcp ? 6 : 17; ip[7] = 64;
      memcpy(ip + 8, s6, 16); memcpy(ip + 24, d6, 16);
    }
    // payload
    for (int k = 0; k < l4len; k++) l4[k] = (uint8_t)R.u32();
    uint16_t sp = (uint16_t)(1024 + R.below(64512)), dp = (uint16_t)(1024 + R.below(64512));
    if (steer_dp >= 0) dp = (uint16_t)steer_dp;
    if (tcp && l4len < 20) tcp = false;  // 64B frames stay UDP
    if (!is6) ip[9] = tcp ? 6 : 17; else ip[6] = tcp ? 6 : 17;
    if (!is6) { put16(ip + 10, 0); put16(ip + 10, csum_fold(sum_bytes(ip, 20))); }
    uint64_t ps = 0;
    if (!is6) { ps += sum_bytes(ip + 12, 8); }
    else { ps += sum_bytes(ip + 8, 32); }
    if (tcp) {
      put16(l4, sp); put16(l4 + 2, dp); put32(l4 + 4, R.u32()); put32(l4 + 8, R.u32());
      l4[12] = 0x50; l4[13] = 0x18; put16(l4 + 14, 8192); put16(l4 + 16, 0); put16(l4 + 18, 0);
      ps += 6 + l4len;
      ps += sum_bytes(l4, l4len);
      put16(l4 + 16, csum_fold(ps));
    } else {
      put16(l4, sp); put16(l4 + 2, dp); put16(l4 + 4, l4len); put16(l4 + 6, 0);
      ps += 17 + l4len;
      ps += sum_bytes(l4, l4len);
      uint16_t ck = csum_fold(ps);
      put16(l4 + 6, ck == 0 ? 0xffff : ck);
    }
    dp_pkt_in_t &pi = w.in[i];
    pi.off = offs[i];
    pi.len = L;
    pi.flags = (overlay && !vxlan) ? DP_IN_SEEDED_OVERLAY : 0;
    pi.iif = 1;
    pi.src_vni = svni;
    w.payload_bytes += L;
  }

  // ---------------- descriptor
  dp_tables_desc_t &d = w.desc;
  d.abi_version = DPGPU_ABI_VERSION;
  d.genid = 1;
  d.fibs = w.fibs.data(); d.n_fibs = (uint32_t)w.fibs.size();
  d.vni_fibs = w.vnis.data(); d.n_vni_fibs = (uint32_t)w.vnis.size();
  d.routes = w.routes.data(); d.n_routes = w.routes.size();
  d.route_nhs = w.nhs.data(); d.n_route_nhs = (uint32_t)w.nhs.size();
  d.entries = w.entries.data(); d.n_entries = (uint32_t)w.entries.size();
  d.instrs = w.instrs.data(); d.n_instrs = (uint32_t)w.instrs.size();
  d.ifaces = w.ifaces.data(); d.n_ifaces = (uint32_t)w.ifaces.size();
  d.adjs = w.adjs.data(); d.n_adjs = (uint32_t)w.adjs.size();
  d.acl_v4 = w.acl4.data(); d.n_acl_v4 = (uint32_t)w.acl4.size();
  d.acl_v6 = w.acl6.data(); d.n_acl_v6 = (uint32_t)w.acl6.size();
  d.acl_defaults = w.acl_def.data(); d.n_acl_defaults = (uint32_t)w.acl_def.size();
  d.ff_remote_v4 = w.ffr4.data(); d.n_ff_remote_v4 = (uint32_t)w.ffr4.size();
  d.ff_local_v4 = w.ffl4.data(); d.n_ff_local_v4 = (uint32_t)w.ffl4.size();
  d.ff_remote_v6 = w.ffr6.data(); d.n_ff_remote_v6 = (uint32_t)w.ffr6.size();
  d.ff_local_v6 = w.ffl6.data(); d.n_ff_local_v6 = (uint32_t)w.ffl6.size();
  d.nat_tables = w.nat_tabs.data(); d.n_nat_tables = (uint32_t)w.nat_tabs.size();
  d.nat_entries = w.nat_ents.data(); d.n_nat_entries = (uint32_t)w.nat_ents.size();
  d.nat_port_ranges = w.nat_prs.data(); d.n_nat_port_ranges = (uint32_t)w.nat_prs.size();
  d.nat_ranges = w.nat_ranges.data(); d.n_nat_ranges = (uint32_t)w.nat_ranges.size();
  *out = W.release();
  return 0;
}

const dp_tables_desc_t *dpw_tables(const dpw_workload_t *w) { return &w->desc; }
uint8_t *dpw_buf(dpw_workload_t *w) { return w->buf.data(); }
uint64_t dpw_buf_bytes(const dpw_workload_t *w) { return w->buf.size(); }
const dp_pkt_in_t *dpw_in(const dpw_workload_t *w) { return w->in.data(); }
uint32_t dpw_n(const dpw_workload_t *w) { return (uint32_t)w->in.size(); }
uint64_t dpw_frame_bytes(const dpw_workload_t *w) { return w->payload_bytes; }

}  // extern "C"

// sizeof of every ABI struct, so the Python ctypes mirror can be checked
extern "C" uint32_t dpw_sizeof(const char *name) {
  struct E { const char *n; uint32_t s; };
  static const E tab[] = {
      {"dp_ipaddr_t", sizeof(dp_ipaddr_t)}, {"dp_prefix_t", sizeof(dp_prefix_t)},
      {"dp_fib_t", sizeof(dp_fib_t)}, {"dp_vni_fib_t", sizeof(dp_vni_fib_t)},
      {"dp_instr_t", sizeof(dp_instr_t)}, {"dp_fib_entry_t", sizeof(dp_fib_entry_t)},
      {"dp_route_nh_t", sizeof(dp_route_nh_t)}, {"dp_route_t", sizeof(dp_route_t)},
      {"dp_iface_t", sizeof(dp_iface_t)}, {"dp_adjacency_t", sizeof(dp_adjacency_t)},
      {"dp_rule_t", sizeof(dp_rule_t)}, {"dp_acl_default_t", sizeof(dp_acl_default_t)},
      {"dp_nat_table_t", sizeof(dp_nat_table_t)}, {"dp_nat_entry_t", sizeof(dp_nat_entry_t)},
      {"dp_port_range_t", sizeof(dp_port_range_t)}, {"dp_nat_range_t", sizeof(dp_nat_range_t)}, {"dp_portfw_rule_t", sizeof(dp_portfw_rule_t)},
      {"dp_masq_expose_t", sizeof(dp_masq_expose_t)}, {"dp_masq_claim_t", sizeof(dp_masq_claim_t)},
      {"dp_acl_key_t", sizeof(dp_acl_key_t)}, {"dp_acl_result_t", sizeof(dp_acl_result_t)},
      {"dp_ff_input_t", sizeof(dp_ff_input_t)}, {"dp_ff_result_t", sizeof(dp_ff_result_t)},
      {"dp_tables_desc_t", sizeof(dp_tables_desc_t)}, {"dp_pkt_in_t", sizeof(dp_pkt_in_t)},
      {"dp_pkt_out_t", sizeof(dp_pkt_out_t)}, {"dp_pkt_meta_t", sizeof(dp_pkt_meta_t)},
      {"dp_flow_key_t", sizeof(dp_flow_key_t)},
      {"dp_flow_t", sizeof(dp_flow_t)}, {"dp_flow_info_t", sizeof(dp_flow_info_t)},
      {"dp_mbuf_layout_t", sizeof(dp_mbuf_layout_t)},
  };
  for (auto &e : tab)
    if (strcmp(e.n, name) == 0) return e.s;
  return 0;
}

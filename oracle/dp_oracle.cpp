// SPDX-License-Identifier: Apache-2.0
//
// TEST INFRASTRUCTURE -- NOT PRODUCT CODE (see dp_oracle.h).
//
// CPU restatement of the reference per-burst packet path.  Structure follows
// the reference on purpose: a parsed `Headers` value with optional layers
// (net/src/headers/mod.rs:67-75), stage functions in pipeline order
// (dataplane/src/packet_processor/mod.rs:130-145), deparse-on-serialize
// (net/src/packet/mod.rs:342-374).  Lookup structures are the simple
// reference ones: binary trie LPM (prefix-trie semantics), linear first-match
// classifiers (acl/src/reference/table.rs:94-101), linear NAT range search.
#include "dp_oracle.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <memory>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// Small helpers
// ---------------------------------------------------------------------------
inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
inline void put16(uint8_t *p, uint16_t v) { p[0] = v >> 8; p[1] = v & 0xff; }
inline void put32(uint8_t *p, uint32_t v) {
  p[0] = v >> 24; p[1] = (v >> 16) & 0xff; p[2] = (v >> 8) & 0xff; p[3] = v & 0xff;
}

struct Ip {  // std::net::IpAddr
  uint8_t fam = 0;  // 4 / 6
  uint8_t b[16] = {0};
  bool operator==(const Ip &o) const {
    return fam == o.fam && memcmp(b, o.b, fam == 4 ? 4 : 16) == 0;
  }
};

inline Ip ip4(const uint8_t *a) { Ip r; r.fam = 4; memcpy(r.b, a, 4); return r; }
inline Ip ip6(const uint8_t *a) { Ip r; r.fam = 6; memcpy(r.b, a, 16); return r; }

inline bool bit_at(const uint8_t *a, int i) { return (a[i >> 3] >> (7 - (i & 7))) & 1; }

// prefix covers address (match-action Prefix::matches semantics,
// match-action/src/predicate.rs:50-53,246-264)
bool prefix_covers(const uint8_t *pfx, int len, const uint8_t *addr) {
  int full = len / 8, rem = len % 8;
  if (memcmp(pfx, addr, full) != 0) return false;
  if (rem) {
    uint8_t m = (uint8_t)(0xff << (8 - rem));
    if ((pfx[full] & m) != (addr[full] & m)) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------
// One's complement checksum (etherparse checksum::Sum16BitWords)
// ---------------------------------------------------------------------------
struct Sum16 {
  uint64_t s = 0;
  void add2(uint8_t a, uint8_t b) { s += (uint32_t)((a << 8) | b); }
  void add_u16(uint16_t v) { s += v; }
  void add_slice(const uint8_t *p, size_t n) {
    size_t i = 0;
    for (; i + 1 < n; i += 2) s += (uint32_t)((p[i] << 8) | p[i + 1]);
    if (i < n) s += (uint32_t)(p[i] << 8);  // odd trailing byte padded with 0
  }
  uint16_t ones_complement() const {
    uint64_t v = s;
    while (v >> 16) v = (v & 0xffff) + (v >> 16);
    return (uint16_t)~v;
  }
};

// ---------------------------------------------------------------------------
// rapidhash-style hash (restatement; parity vs reference UNPINNED,
// rapidhash 4.5.1 over Rust `Hash` encodings)
// ---------------------------------------------------------------------------
const uint64_t kSecret[3] = {0x2d358dccaa6c78a5ull, 0x8bb84b93962eacc9ull,
                             0x4b33a62ed433d4a3ull};
const uint64_t kSeed = 0xbdd89aa982704029ull;
inline void mum(uint64_t *a, uint64_t *b) {
  unsigned __int128 r = (unsigned __int128)(*a) * (*b);
  *a = (uint64_t)r;
  *b = (uint64_t)(r >> 64);
}
inline uint64_t mix(uint64_t a, uint64_t b) { mum(&a, &b); return a ^ b; }
inline uint64_t r64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
inline uint64_t r32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

uint64_t rapid(const uint8_t *p, size_t len) {
  uint64_t seed = kSeed;
  seed ^= mix(seed ^ kSecret[0], kSecret[1]) ^ len;
  uint64_t a, b;
  if (len <= 16) {
    if (len >= 4) {
      const uint8_t *plast = p + len - 4;
      a = (r32(p) << 32) | r32(plast);
      const uint64_t delta = ((len & 24) >> (len >> 3));
      b = (r32(p + delta) << 32) | r32(plast - delta);
    } else if (len > 0) {
      a = ((uint64_t)p[0] << 56) | ((uint64_t)p[len >> 1] << 32) | p[len - 1];
      b = 0;
    } else {
      a = b = 0;
    }
  } else {
    size_t i = len;
    if (i > 48) {
      uint64_t see1 = seed, see2 = seed;
      while (i >= 48) {
        seed = mix(r64(p) ^ kSecret[0], r64(p + 8) ^ seed);
        see1 = mix(r64(p + 16) ^ kSecret[1], r64(p + 24) ^ see1);
        see2 = mix(r64(p + 32) ^ kSecret[2], r64(p + 40) ^ see2);
        p += 48;
        i -= 48;
      }
      seed ^= see1 ^ see2;
    }
    if (i > 16) {
      seed = mix(r64(p) ^ kSecret[2], r64(p + 8) ^ seed ^ kSecret[1]);
      if (i > 32) seed = mix(r64(p + 16) ^ kSecret[2], r64(p + 24) ^ seed);
    }
    a = r64(p + i - 16);
    b = r64(p + i - 8);
  }
  a ^= kSecret[1];
  b ^= seed;
  mum(&a, &b);
  return mix(a ^ kSecret[0] ^ len, b ^ kSecret[1]);
}

// ---------------------------------------------------------------------------
// Parsed headers (net/src/headers/mod.rs:67-75)
// ---------------------------------------------------------------------------
enum L4Kind { L4_NONE = 0, L4_TCP, L4_UDP, L4_ICMP4, L4_ICMP6 };
enum ExtKind { EXT_RAW = 0, EXT_FRAG, EXT_AUTH };

struct Eth {  // etherparse Ethernet2Header
  uint8_t dst[6], src[6];
  uint16_t type;
};
struct Vlan {  // etherparse SingleVlanHeader: round-trips exactly
  uint16_t tci, inner;
  uint16_t vid() const { return tci & 0x0fff; }
};
struct Ipv4 {  // etherparse Ipv4Header (no reserved flag bit: dropped on deparse)
  uint8_t dscp, ecn;
  uint16_t total_len, id;
  bool df, mf;
  uint16_t frag;
  uint8_t ttl, proto;
  uint16_t csum;
  uint8_t src[4], dst[4];
  uint8_t opts[40];
  uint8_t opt_len;
  int hlen() const { return 20 + opt_len; }
};
struct Ipv6 {
  uint8_t tc;
  uint32_t flow;
  uint16_t plen;
  uint8_t nh, hop;
  uint8_t src[16], dst[16];
};
struct Ext {  // HopByHop/DestOpts/Routing raw, Fragment, Auth (normalized bytes)
  int kind;
  uint8_t nh;
  std::vector<uint8_t> bytes;
};
struct Tcp {  // etherparse TcpHeader: reserved bits dropped on deparse
  uint16_t sport, dport;
  uint32_t seq, ack;
  uint8_t doff;
  bool ns;
  uint8_t flags;
  uint16_t win, csum, urg;
  uint8_t opts[40];
  int hlen() const { return doff * 4; }
};
struct Udp {
  uint16_t sport, dport, len, csum;
};
struct Icmp {  // type, code, checksum, rest (4 or 16 bytes)
  uint8_t raw[20];
  int hlen;
};

// EmbeddedHeaders (net/src/headers/embedded.rs:43-48): the IP packet fragment
// an ICMP error message carries -- IP header, <= MAX_NET_EXTENSIONS extension
// headers, and a possibly truncated transport header (TruncatedTcp/Udp/
// Icmp4/Icmp6: a full header, or a partial one that keeps every remaining
// byte, tcp/truncated.rs:67-103, udp/truncated.rs:67-103, icmp4/truncated.rs).
struct Emb {
  bool present = false;
  int net = 0;  // 4 / 6
  Ipv4 v4{};
  Ipv6 v6{};
  std::vector<Ext> ext;
  int tk = L4_NONE;  // transport kind (L4_*), L4_NONE: none
  bool full = false;
  Tcp tcp{};
  Udp udp{};
  Icmp icmp{};
  std::vector<uint8_t> part;  // partial transport header bytes (deparsed as they are)
  int net_size() const { return net == 4 ? v4.hlen() : net == 6 ? 40 : 0; }
  int transport_size() const {
    if (tk == L4_NONE) return 0;
    if (!full) return (int)part.size();
    return tk == L4_TCP ? tcp.hlen() : tk == L4_UDP ? 8 : icmp.hlen;
  }
  int size() const {  // EmbeddedHeaders::size (embedded.rs:402-414)
    int s = net_size() + transport_size();
    if (net) for (auto &e : ext) s += (int)e.bytes.size();
    return s;
  }
};

struct Headers {
  bool has_eth = false;
  Eth eth{};
  std::vector<Vlan> vlans;
  int net = 0;  // 0 none, 4, 6
  Ipv4 v4{};
  Ipv6 v6{};
  std::vector<Ext> ext;
  int l4 = L4_NONE;
  Tcp tcp{};
  Udp udp{};
  Icmp icmp{};
  bool has_vxlan = false;
  uint32_t vni = 0;
  Emb emb;  // Headers::embedded_ip (ICMP error messages only)

  int size() const {
    int s = has_eth ? 14 : 0;
    s += 4 * (int)vlans.size();
    if (net == 4) s += v4.hlen();
    if (net == 6) s += 40;
    if (net) for (auto &e : ext) s += (int)e.bytes.size();
    if (net && l4 == L4_TCP) s += tcp.hlen();
    if (net && l4 == L4_UDP) s += 8;
    if (net && (l4 == L4_ICMP4 || l4 == L4_ICMP6)) s += icmp.hlen;
    if (net && l4 != L4_NONE && has_vxlan) s += 8;
    if (emb.present) s += emb.size();
    return s;
  }
};

struct Meta {
  int done = -1;  // DoneReason or -1 (None)
  uint32_t flags = DP_META_INITIALIZED | DP_META_KEEP;
  bool has_vrf = false;
  uint32_t vrf = 0;
  uint32_t src_vni = 0, dst_vni = 0;  // 0 = None
  bool has_oif = false;
  uint32_t oif = 0;
  bool has_nh = false;
  Ip nh;
  bool has_dscp = false;
  uint8_t dscp = 0, ecn = 0;
  uint32_t fib_entry = UINT32_MAX;
  uint32_t acl_rule = UINT32_MAX;
  uint8_t acl = 0;
};

// FlowKey (net/src/flows/flow_key.rs:457-463) as a comparable value.  Its Hash
// covers (src_vpcd, src_ip, src_port, dst_ip, dst_port) and its Eq the whole
// key; the TCP/UDP port Eq is symmetric (flow_key.rs:57-60, 123-127) but a
// port-swapped key hashes elsewhere, so a lookup matches the key exactly.
struct FKey {
  uint32_t vni = 0;
  uint8_t fam = 0, kind = 0;
  uint16_t sp = 0, dp = 0;
  uint8_t src[16] = {0}, dst[16] = {0};
  bool operator==(const FKey &o) const {
    return vni == o.vni && fam == o.fam && kind == o.kind && sp == o.sp && dp == o.dp &&
           memcmp(src, o.src, 16) == 0 && memcmp(dst, o.dst, 16) == 0;
  }
};
struct FKeyHash {
  size_t operator()(const FKey &k) const {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {
      for (size_t i = 0; i < n; i++) { h ^= ((const uint8_t *)p)[i]; h *= 1099511628211ull; }
    };
    mix(&k.vni, 4); mix(&k.fam, 1); mix(&k.kind, 1); mix(&k.sp, 2); mix(&k.dp, 2);
    mix(k.src, 16); mix(k.dst, 16);
    return (size_t)h;
  }
};
struct Packet {
  Headers h;
  uint8_t *buf;
  uint64_t pay_start, pay_end;  // payload is buf[pay_start, pay_end)
  uint64_t room_start;          // first byte this packet may write
  Meta m;
  int64_t flow = -1;            // PacketMeta.flow_info (a flow of the oracle's table)
  bool has_ikey = false;        // PacketMeta.flow_key: the key before static NAT
  FKey ikey;                    // (flow-filter/src/lib.rs:193-201)
  void done(int r) { if (m.done < 0) m.done = r; }
  void done_force(int r) { m.done = r; }
  bool is_done() const { return m.done >= 0; }
  bool overlay() const { return m.flags & DP_META_IS_OVERLAY; }
};

// ---------------------------------------------------------------------------
// Parse (Headers::parse, net/src/headers/mod.rs:474-578)
// ---------------------------------------------------------------------------
struct Reader {
  const uint8_t *p;
  size_t len, pos;
  size_t remaining() const { return len - pos; }
  const uint8_t *cur() const { return p + pos; }
};

// Eth::parse (net/src/eth/mod.rs:111-146): dst != 0, src != 0 && !multicast
bool parse_eth(Reader &r, Eth &e) {
  if (r.remaining() < 14) return false;
  const uint8_t *q = r.cur();
  memcpy(e.dst, q, 6);
  memcpy(e.src, q + 6, 6);
  e.type = be16(q + 12);
  static const uint8_t zero[6] = {0};
  if (memcmp(e.dst, zero, 6) == 0) return false;
  if (memcmp(e.src, zero, 6) == 0) return false;
  if (e.src[0] & 1) return false;
  r.pos += 14;
  return true;
}

// Vlan::parse (net/src/vlan/mod.rs:327-354); Vid 0 and 4095 invalid (:74-81)
bool parse_vlan(Reader &r, Vlan &v) {
  if (r.remaining() < 4) return false;
  const uint8_t *q = r.cur();
  v.tci = be16(q);
  v.inner = be16(q + 2);
  uint16_t vid = v.tci & 0x0fff;
  if (vid == 0 || vid == 4095) return false;
  r.pos += 4;
  return true;
}

// Ipv4::parse (net/src/ipv4/mod.rs:351-373) over etherparse
// Ipv4HeaderSlice::from_slice: version 4, ihl >= 5, len >= ihl*4,
// total_len >= ihl*4; then source must be unicast (not multicast/broadcast).
bool parse_ipv4(Reader &r, Ipv4 &h) {
  if (r.remaining() < 20) return false;
  const uint8_t *q = r.cur();
  if ((q[0] >> 4) != 4) return false;
  int ihl = q[0] & 0xf;
  if (ihl < 5) return false;
  int hlen = ihl * 4;
  if ((int)r.remaining() < hlen) return false;
  uint16_t total = be16(q + 2);
  if (total < hlen) return false;
  h.dscp = q[1] >> 2;
  h.ecn = q[1] & 3;
  h.total_len = total;
  h.id = be16(q + 4);
  h.df = (q[6] >> 6) & 1;
  h.mf = (q[6] >> 5) & 1;
  h.frag = (uint16_t)(((q[6] & 0x1f) << 8) | q[7]);
  h.ttl = q[8];
  h.proto = q[9];
  h.csum = be16(q + 10);
  memcpy(h.src, q + 12, 4);
  memcpy(h.dst, q + 16, 4);
  h.opt_len = (uint8_t)(hlen - 20);
  memcpy(h.opts, q + 20, h.opt_len);
  // UnicastIpv4Addr::new: not multicast (224/4) and not broadcast
  if ((h.src[0] & 0xf0) == 0xe0) return false;
  if (h.src[0] == 255 && h.src[1] == 255 && h.src[2] == 255 && h.src[3] == 255) return false;
  r.pos += hlen;
  return true;
}

// Ipv6::parse (net/src/ipv6/mod.rs:309-335): version 6, src not multicast
bool parse_ipv6(Reader &r, Ipv6 &h) {
  if (r.remaining() < 40) return false;
  const uint8_t *q = r.cur();
  if ((q[0] >> 4) != 6) return false;
  h.tc = (uint8_t)(((q[0] & 0xf) << 4) | (q[1] >> 4));
  h.flow = ((uint32_t)(q[1] & 0xf) << 16) | ((uint32_t)q[2] << 8) | q[3];
  h.plen = be16(q + 4);
  h.nh = q[6];
  h.hop = q[7];
  memcpy(h.src, q + 8, 16);
  memcpy(h.dst, q + 24, 16);
  if (h.src[0] == 0xff) return false;
  r.pos += 40;
  return true;
}

// Ipv6RawExtHeader (HopByHop 0 / Routing 43 / DestOpts 60): (len+1)*8 bytes
bool parse_ext_raw(Reader &r, Ext &e) {
  if (r.remaining() < 8) return false;
  const uint8_t *q = r.cur();
  size_t n = ((size_t)q[1] + 1) * 8;
  if (r.remaining() < n) return false;
  e.kind = EXT_RAW;
  e.nh = q[0];
  e.bytes.assign(q, q + n);
  r.pos += n;
  return true;
}
// Ipv6FragmentHeader (44): 8 bytes; reserved bits not kept by etherparse
bool parse_ext_frag(Reader &r, Ext &e) {
  if (r.remaining() < 8) return false;
  const uint8_t *q = r.cur();
  e.kind = EXT_FRAG;
  e.nh = q[0];
  e.bytes.assign(q, q + 8);
  e.bytes[1] = 0;                        // reserved
  e.bytes[3] = (uint8_t)(q[3] & 0xf9);   // res bits 1-2 zeroed, M kept
  r.pos += 8;
  return true;
}
// IpAuthHeader (51): (payload_len+2)*4 bytes, payload_len >= 1; reserved zeroed
bool parse_ext_auth(Reader &r, Ext &e) {
  if (r.remaining() < 12) return false;
  const uint8_t *q = r.cur();
  if (q[1] == 0) return false;
  size_t n = ((size_t)q[1] + 2) * 4;
  if (r.remaining() < n) return false;
  e.kind = EXT_AUTH;
  e.nh = q[0];
  e.bytes.assign(q, q + n);
  e.bytes[2] = 0;
  e.bytes[3] = 0;
  r.pos += n;
  return true;
}

// Tcp::parse (net/src/tcp/mod.rs:330-365)
bool parse_tcp(Reader &r, Tcp &t) {
  if (r.remaining() < 20) return false;
  const uint8_t *q = r.cur();
  int doff = q[12] >> 4;
  if (doff < 5) return false;
  if ((int)r.remaining() < doff * 4) return false;
  t.sport = be16(q);
  t.dport = be16(q + 2);
  if (t.sport == 0 || t.dport == 0) return false;
  t.seq = be32(q + 4);
  t.ack = be32(q + 8);
  t.doff = (uint8_t)doff;
  t.ns = q[12] & 1;
  t.flags = q[13];
  t.win = be16(q + 14);
  t.csum = be16(q + 16);
  t.urg = be16(q + 18);
  memcpy(t.opts, q + 20, doff * 4 - 20);
  r.pos += doff * 4;
  return true;
}

// Udp::parse (net/src/udp/mod.rs:180-211)
bool parse_udp(Reader &r, Udp &u) {
  if (r.remaining() < 8) return false;
  const uint8_t *q = r.cur();
  u.sport = be16(q);
  u.dport = be16(q + 2);
  u.len = be16(q + 4);
  u.csum = be16(q + 6);
  if (u.sport == 0 || u.dport == 0) return false;
  r.pos += 8;
  return true;
}

// Icmpv4Header / Icmpv6Header: 8 bytes (v4 timestamp request/reply: 20)
bool parse_icmp(Reader &r, Icmp &ic, bool v6) {
  if (r.remaining() < 8) return false;
  const uint8_t *q = r.cur();
  int n = 8;
  if (!v6 && (q[0] == 13 || q[0] == 14) && q[1] == 0) n = 20;
  if ((int)r.remaining() < n) return false;
  memcpy(ic.raw, q, n);
  ic.hlen = n;
  r.pos += n;
  return true;
}

// --- ICMP types as the reference sees them ---------------------------------
// etherparse 0.21 decodes the type/code pair (Icmpv4Type / Icmpv6Type); a
// pair it does not know is Unknown.  The reference maps that onto its own
// enums (net/src/icmp4/mod.rs:406-465, net/src/icmp6/mod.rs:396-459), which
// also turn a Redirect with a non-unicast gateway and a Packet Too Big with
// an MTU below 1280 into Unknown.  Error messages: icmp4/mod.rs:555-563,
// icmp6/mod.rs:577-585.
bool icmp4_error(const uint8_t *q) {
  const uint8_t t = q[0], c = q[1];
  switch (t) {
    case 3: return c <= 15;   // DestUnreachable (16 codes)
    case 5: {                 // Redirect (4 codes), gateway UnicastIpv4Addr
      if (c > 3) return false;
      const bool bcast = q[4] == 255 && q[5] == 255 && q[6] == 255 && q[7] == 255;
      return !((q[4] & 0xf0) == 0xe0 || bcast);
    }
    case 11: return c <= 1;   // TimeExceeded
    case 12: return c <= 2;   // ParameterProblem
    default: return false;
  }
}
bool icmp6_error(const uint8_t *q) {
  const uint8_t t = q[0], c = q[1];
  switch (t) {
    case 1: return c <= 6;                      // DestUnreachable
    case 2: return c == 0 && be32(q + 4) >= 1280;  // PacketTooBig (Icmp6PacketTooBig::new)
    case 3: return c <= 1;                      // TimeExceeded
    case 4: return c <= 10;                     // ParameterProblem
    default: return false;
  }
}
// The 8 (v4 timestamp: 20) header bytes Icmpv4Header / Icmpv6Header write
// back (to_bytes): an error message keeps only the fields its type defines
// (v4 DestUnreachable: the next-hop MTU of code 4; Redirect: the gateway;
// ParameterProblem code 0: the pointer byte; v6 PacketTooBig: the MTU,
// ParameterProblem: the pointer), the unused bytes -- RFC 4884's length
// among them -- are written as zero.  Other types are written back as parsed.
void icmp_norm(const uint8_t *q, int hlen, bool v6, uint8_t *o) {
  memcpy(o, q, hlen);
  if (!v6 && icmp4_error(q)) {
    if (q[0] == 3) { o[4] = o[5] = 0; if (q[1] != 4) o[6] = o[7] = 0; }
    if (q[0] == 11) o[4] = o[5] = o[6] = o[7] = 0;
    if (q[0] == 12) { o[5] = o[6] = o[7] = 0; if (q[1] != 0) o[4] = 0; }
  }
  if (v6 && icmp6_error(q)) {
    if (q[0] == 1 || q[0] == 3) o[4] = o[5] = o[6] = o[7] = 0;
  }
}
// Icmp4::identifier / Icmp6::identifier of a full header: decoded echo and
// timestamp messages (code 0) carry one (icmp4/mod.rs:565-576)
bool icmp_full_identifier(const Icmp &ic, bool v6, uint16_t &id) {
  const uint8_t t = ic.raw[0], c = ic.raw[1];
  const bool q = v6 ? ((t == 128 || t == 129) && c == 0)
                    : ((t == 0 || t == 8 || t == 13 || t == 14) && c == 0);
  if (!q) return false;
  id = be16(ic.raw + 4);
  return true;
}

// TruncatedTcp::parse (tcp/truncated.rs:193-214): the full header if
// Tcp::parse succeeds; a Length error (fewer bytes than the header) gives a
// partial header of every remaining byte (>= 4, non-zero ports); any other
// error (data offset < 5, zero port) fails.
bool parse_trunc_tcp(Reader &r, Emb &e) {
  const size_t n = r.remaining();
  const uint8_t *q = r.cur();
  bool len_err = n < 20;
  if (!len_err) {
    const int doff = q[12] >> 4;
    if (doff < 5) return false;
    len_err = n < (size_t)doff * 4;
  }
  if (!len_err) {
    if (!parse_tcp(r, e.tcp)) return false;  // zero ports
    e.tk = L4_TCP; e.full = true;
    return true;
  }
  if (n < 4 || be16(q) == 0 || be16(q + 2) == 0) return false;
  e.tk = L4_TCP; e.full = false;
  e.part.assign(q, q + n);
  r.pos += n;
  return true;
}
// TruncatedUdp::parse (udp/truncated.rs): full >= 8 bytes, else partial (>= 4)
bool parse_trunc_udp(Reader &r, Emb &e) {
  const size_t n = r.remaining();
  const uint8_t *q = r.cur();
  if (n >= 8) {
    if (!parse_udp(r, e.udp)) return false;
    e.tk = L4_UDP; e.full = true;
    return true;
  }
  if (n < 4 || be16(q) == 0 || be16(q + 2) == 0) return false;
  e.tk = L4_UDP; e.full = false;
  e.part.assign(q, q + n);
  r.pos += n;
  return true;
}
// TruncatedIcmp4 / TruncatedIcmp6::parse (icmp4/truncated.rs:200-221): the
// full header (8 bytes, v4 timestamp 20), else a partial one (>= 2 bytes)
bool parse_trunc_icmp(Reader &r, Emb &e, bool v6) {
  const size_t n = r.remaining();
  const uint8_t *q = r.cur();
  e.tk = v6 ? L4_ICMP6 : L4_ICMP4;
  if (parse_icmp(r, e.icmp, v6)) { e.full = true; return true; }
  if (n < 2) { e.tk = L4_NONE; return false; }
  e.full = false;
  e.part.assign(q, q + n);
  r.pos += n;
  return true;
}

// EmbeddedHeaders::parse_with (net/src/headers/embedded.rs:289-397): the IP
// header, then Ipv4::parse_embedded_payload / Ipv6::parse_embedded_payload
// (ipv4/mod.rs:320-331, ipv6/mod.rs:266-287, ipv6/ext_parse.rs:46-69,
// ip_auth/v4.rs:67-87) with the MAX_NET_EXTENSIONS quirk of the main loop.
// Returns the consumed bytes, or -1 when the IP header does not parse (no
// embedded headers at all, icmp4/mod.rs:626-646).
int parse_embedded(const uint8_t *p, size_t len, bool v6, Emb &e) {
  Reader r{p, len, 0};
  e = Emb{};
  if (!v6) { if (!parse_ipv4(r, e.v4)) return -1; e.net = 4; }
  else { if (!parse_ipv6(r, e.v6)) return -1; e.net = 6; }
  e.present = true;
  // the loop of embedded.rs:318-390: parse the header after `prior`
  // (consuming it), then record `prior` -- an extension header past the limit
  // breaks the loop after its successor was consumed
  enum { P_IP, P_EXT, P_TR };
  int prior = P_IP;
  Ext pext{};
  uint8_t nh = v6 ? e.v6.nh : e.v4.proto;
  Emb tr;  // a parsed transport, recorded when it becomes `prior`
  for (;;) {
    int next = -1;
    Ext x{};
    if (prior != P_TR) {
      bool ok = false;
      switch (nh) {
        case 6: ok = parse_trunc_tcp(r, tr); next = P_TR; break;
        case 17: ok = parse_trunc_udp(r, tr); next = P_TR; break;
        case 1: if (!v6) { ok = parse_trunc_icmp(r, tr, false); next = P_TR; } break;
        case 58: if (v6) { ok = parse_trunc_icmp(r, tr, true); next = P_TR; } break;
        case 51: ok = parse_ext_auth(r, x); next = P_EXT; break;
        case 0: case 43: case 60: if (v6) { ok = parse_ext_raw(r, x); next = P_EXT; } break;
        case 44: if (v6) { ok = parse_ext_frag(r, x); next = P_EXT; } break;
        default: break;
      }
      if (!ok) next = -1;
    }
    bool brk = false;
    if (prior == P_EXT) {
      if (e.ext.size() < 3) e.ext.push_back(pext);
      else brk = true;
    } else if (prior == P_TR) {
      e.tk = tr.tk; e.full = tr.full; e.tcp = tr.tcp; e.udp = tr.udp; e.icmp = tr.icmp;
      e.part = tr.part;
    }
    if (brk || next < 0) break;
    prior = next;
    if (next == P_EXT) { pext = x; nh = x.nh; }
  }
  return (int)r.pos;
}

// Vxlan::parse (net/src/vxlan/mod.rs:91-122)
bool parse_vxlan(Reader &r, uint32_t &vni) {
  if (r.remaining() < 8) return false;
  const uint8_t *q = r.cur();
  if ((q[0] & 0x08) != 0x08) return false;
  if (q[1] || q[2] || q[3] || q[7]) return false;
  uint32_t v = ((uint32_t)q[4] << 16) | ((uint32_t)q[5] << 8) | q[6];
  if (v == 0) return false;
  vni = v;
  r.pos += 8;
  return true;
}

// Headers::parse loop, including its MAX_VLANS / MAX_NET_EXTENSIONS quirk:
// the header after the limit is still consumed but not recorded.
// Returns consumed bytes, or -1 on Eth failure.
enum HKind { H_ETH, H_VLAN, H_V4, H_V6, H_EXT, H_TCP, H_UDP, H_ICMP4, H_ICMP6, H_VXLAN, H_EMB };
struct HeaderVal {
  int kind;
  Vlan vlan;
  Ipv4 v4;
  Ipv6 v6;
  Ext ext;
  Tcp tcp;
  Udp udp;
  Icmp icmp;
  uint32_t vni;
  Emb emb;
};

bool parse_by_ethertype(uint16_t et, Reader &r, HeaderVal &out) {
  switch (et) {
    case 0x0800: out.kind = H_V4; return parse_ipv4(r, out.v4);
    case 0x86dd: out.kind = H_V6; return parse_ipv6(r, out.v6);
    case 0x8100: case 0x9100: case 0x88a8: out.kind = H_VLAN; return parse_vlan(r, out.vlan);
    default: return false;
  }
}

bool parse_by_proto(uint8_t proto, bool v6_ctx, bool v4_ctx, Reader &r, HeaderVal &out) {
  switch (proto) {
    case 6: out.kind = H_TCP; return parse_tcp(r, out.tcp);
    case 17: out.kind = H_UDP; return parse_udp(r, out.udp);
    case 1:
      if (!v4_ctx) return false;
      out.kind = H_ICMP4; return parse_icmp(r, out.icmp, false);
    case 58:
      if (!v6_ctx) return false;
      out.kind = H_ICMP6; return parse_icmp(r, out.icmp, true);
    case 51: out.kind = H_EXT; return parse_ext_auth(r, out.ext);
    case 0: if (!v6_ctx) return false; out.kind = H_EXT; return parse_ext_raw(r, out.ext);
    case 43: if (!v6_ctx) return false; out.kind = H_EXT; return parse_ext_raw(r, out.ext);
    case 60: if (!v6_ctx) return false; out.kind = H_EXT; return parse_ext_raw(r, out.ext);
    case 44: if (!v6_ctx) return false; out.kind = H_EXT; return parse_ext_frag(r, out.ext);
    default: return false;
  }
}

// The v4/v6 context of an AH header: Ipv4Auth parses v4 payload protocols
// (TCP/UDP/ICMP/AH), Ipv6Auth the v6 ones (net/src/ip_auth/v4.rs:42-60).
bool parse_next_ctx(const HeaderVal &prior, Reader &r, HeaderVal &out, bool v6ctx) {
  switch (prior.kind) {
    case H_ETH: return false;  // handled by caller
    case H_VLAN: return parse_by_ethertype(prior.vlan.inner, r, out);
    case H_V4: return parse_by_proto(prior.v4.proto, false, true, r, out);
    case H_V6: return parse_by_proto(prior.v6.nh, true, false, r, out);
    case H_EXT: {
      // Ipv4Auth::parse_payload: TCP/UDP/ICMP/AH only (net/src/ip_auth)
      uint8_t nh = prior.ext.nh;
      if (!v6ctx) {
        if (nh == 6 || nh == 17 || nh == 1 || nh == 51) return parse_by_proto(nh, false, true, r, out);
        return false;
      }
      return parse_by_proto(nh, true, false, r, out);  // ext_parse.rs dispatch
    }
    case H_ICMP4:
    case H_ICMP6: {
      // Icmp4/Icmp6::parse_payload (icmp4/mod.rs:626-646): an error message's
      // embedded packet fragment
      const bool v6 = prior.kind == H_ICMP6;
      if (!(v6 ? icmp6_error(prior.icmp.raw) : icmp4_error(prior.icmp.raw))) return false;
      const int c = parse_embedded(r.cur(), r.remaining(), v6, out.emb);
      if (c < 0) return false;
      out.kind = H_EMB;
      r.pos += (size_t)c;
      return true;
    }
    case H_UDP:
      // Udp::parse_payload: VXLAN only on dport 4789 (net/src/udp/mod.rs:152-166)
      if (prior.udp.dport == 4789) {
        out.kind = H_VXLAN;
        return parse_vxlan(r, out.vni);
      }
      return false;
    default:
      // TCP / VXLAN / embedded headers: no further parse
      return false;
  }
}

int parse_headers(const uint8_t *p, size_t len, Headers &h) {
  Reader r{p, len, 0};
  if (len > 65535) return -1;
  if (!parse_eth(r, h.eth)) return -1;
  h.has_eth = true;
  HeaderVal prior{};
  // first hop after Eth
  HeaderVal nxt{};
  bool ok = parse_by_ethertype(h.eth.type, r, nxt);
  bool v6ctx = false;
  if (!ok) return (int)r.pos;
  prior = nxt;
  for (;;) {
    HeaderVal next{};
    bool have_next = parse_next_ctx(prior, r, next, v6ctx);
    bool brk = false;
    switch (prior.kind) {
      case H_V4: h.net = 4; h.v4 = prior.v4; v6ctx = false; break;
      case H_V6: h.net = 6; h.v6 = prior.v6; v6ctx = true; break;
      case H_TCP: h.l4 = L4_TCP; h.tcp = prior.tcp; break;
      case H_UDP: h.l4 = L4_UDP; h.udp = prior.udp; break;
      case H_ICMP4: h.l4 = L4_ICMP4; h.icmp = prior.icmp; break;
      case H_ICMP6: h.l4 = L4_ICMP6; h.icmp = prior.icmp; break;
      case H_VXLAN: h.has_vxlan = true; h.vni = prior.vni; break;
      case H_EMB: h.emb = prior.emb; break;
      case H_VLAN:
        if (h.vlans.size() < 4) h.vlans.push_back(prior.vlan); else brk = true;
        break;
      case H_EXT:
        if (h.ext.size() < 3) h.ext.push_back(prior.ext); else brk = true;
        break;
    }
    if (brk || !have_next) break;
    prior = next;
  }
  return (int)r.pos;
}

// ---------------------------------------------------------------------------
// Deparse (Headers::deparse, net/src/headers/mod.rs:617-691)
// ---------------------------------------------------------------------------
int deparse_ipv4(const Ipv4 &h, uint8_t *q) {
  int hl = h.hlen();
  q[0] = (uint8_t)(0x40 | (hl / 4));
  q[1] = (uint8_t)((h.dscp << 2) | h.ecn);
  put16(q + 2, h.total_len);
  put16(q + 4, h.id);
  q[6] = (uint8_t)((h.df ? 0x40 : 0) | (h.mf ? 0x20 : 0) | ((h.frag >> 8) & 0x1f));
  q[7] = h.frag & 0xff;
  q[8] = h.ttl;
  q[9] = h.proto;
  put16(q + 10, h.csum);
  memcpy(q + 12, h.src, 4);
  memcpy(q + 16, h.dst, 4);
  memcpy(q + 20, h.opts, h.opt_len);
  return hl;
}

// etherparse Ipv4Header::calc_header_checksum (no 0 -> 0xffff mapping)
uint16_t ipv4_checksum(const Ipv4 &h) {
  uint8_t tmp[60];
  Ipv4 c = h;
  c.csum = 0;
  int n = deparse_ipv4(c, tmp);
  Sum16 s;
  s.add_slice(tmp, n);
  return s.ones_complement();
}

int deparse_ipv6(const Ipv6 &h, uint8_t *q) {
  q[0] = (uint8_t)(0x60 | (h.tc >> 4));
  q[1] = (uint8_t)(((h.tc & 0xf) << 4) | ((h.flow >> 16) & 0xf));
  q[2] = (h.flow >> 8) & 0xff;
  q[3] = h.flow & 0xff;
  put16(q + 4, h.plen);
  q[6] = h.nh;
  q[7] = h.hop;
  memcpy(q + 8, h.src, 16);
  memcpy(q + 24, h.dst, 16);
  return 40;
}

int deparse_tcp(const Tcp &t, uint8_t *q) {
  put16(q, t.sport);
  put16(q + 2, t.dport);
  put32(q + 4, t.seq);
  put32(q + 8, t.ack);
  q[12] = (uint8_t)((t.doff << 4) | (t.ns ? 1 : 0));
  q[13] = t.flags;
  put16(q + 14, t.win);
  put16(q + 16, t.csum);
  put16(q + 18, t.urg);
  memcpy(q + 20, t.opts, t.hlen() - 20);
  return t.hlen();
}

int deparse_icmp(const Icmp &ic, bool v6, uint8_t *q) {
  icmp_norm(ic.raw, ic.hlen, v6, q);
  return ic.hlen;
}
// EmbeddedHeaders::deparse pieces (embedded.rs:416-461): the IP header, the
// extension headers, the transport header (a partial one as parsed)
int deparse_emb_ip(const Emb &e, uint8_t *q) {
  return e.net == 4 ? deparse_ipv4(e.v4, q) : deparse_ipv6(e.v6, q);
}
int deparse_emb_transport(const Emb &e, uint8_t *q) {
  if (e.tk == L4_NONE) return 0;
  if (!e.full) { memcpy(q, e.part.data(), e.part.size()); return (int)e.part.size(); }
  switch (e.tk) {
    case L4_TCP: return deparse_tcp(e.tcp, q);
    case L4_UDP:
      put16(q, e.udp.sport); put16(q + 2, e.udp.dport); put16(q + 4, e.udp.len); put16(q + 6, e.udp.csum);
      return 8;
    default: return deparse_icmp(e.icmp, e.tk == L4_ICMP6, q);
  }
}
int deparse_emb(const Emb &e, uint8_t *q) {
  int o = deparse_emb_ip(e, q);
  for (auto &x : e.ext) { memcpy(q + o, x.bytes.data(), x.bytes.size()); o += (int)x.bytes.size(); }
  return o + deparse_emb_transport(e, q + o);
}
// icmp_any/checksum.rs:226-259 get_payload_for_checksum: the embedded IP
// header, the embedded transport header, then the payload -- the embedded
// extension headers are not part of it (as in the reference)
std::vector<uint8_t> icmp_checksum_payload(const Emb &e, const uint8_t *pay, size_t plen) {
  std::vector<uint8_t> v(e.net_size() + e.transport_size() + plen);
  int o = deparse_emb_ip(e, v.data());
  o += deparse_emb_transport(e, v.data() + o);
  if (plen) memcpy(v.data() + o, pay, plen);
  return v;
}
// Icmpv4Type::calc_checksum / Icmpv6Type::calc_checksum over the header as
// written back and `pay` (v6: pseudo header of the outer IPv6 addresses)
uint16_t icmp_checksum(const Headers &h, const uint8_t *pay, size_t plen) {
  const bool v6 = h.l4 == L4_ICMP6;
  uint8_t hb[20];
  icmp_norm(h.icmp.raw, h.icmp.hlen, v6, hb);
  hb[2] = hb[3] = 0;
  Sum16 s;
  if (v6) {
    uint32_t tl = (uint32_t)h.icmp.hlen + (uint32_t)plen;
    s.add_slice(h.v6.src, 16); s.add_slice(h.v6.dst, 16);
    s.add_u16((uint16_t)(tl >> 16)); s.add_u16((uint16_t)tl); s.add2(0, 0); s.add2(0, 58);
  }
  s.add_slice(hb, h.icmp.hlen);
  s.add_slice(pay, plen);
  return s.ones_complement();
}
bool icmp_is_error_msg(const Headers &h) {
  if (h.l4 == L4_ICMP4) return icmp4_error(h.icmp.raw);
  if (h.l4 == L4_ICMP6) return icmp6_error(h.icmp.raw);
  return false;
}

int deparse_headers(const Headers &h, uint8_t *q) {
  int o = 0;
  if (h.has_eth) {
    memcpy(q, h.eth.dst, 6);
    memcpy(q + 6, h.eth.src, 6);
    put16(q + 12, h.eth.type);
    o = 14;
  }
  for (auto &v : h.vlans) {
    put16(q + o, v.tci);
    put16(q + o + 2, v.inner);
    o += 4;
  }
  if (h.net == 0) return o;
  if (h.net == 4) o += deparse_ipv4(h.v4, q + o);
  else o += deparse_ipv6(h.v6, q + o);
  for (auto &e : h.ext) {
    memcpy(q + o, e.bytes.data(), e.bytes.size());
    o += (int)e.bytes.size();
  }
  switch (h.l4) {
    case L4_NONE: return o;
    case L4_TCP: o += deparse_tcp(h.tcp, q + o); break;
    case L4_UDP:
      put16(q + o, h.udp.sport); put16(q + o + 2, h.udp.dport);
      put16(q + o + 4, h.udp.len); put16(q + o + 6, h.udp.csum);
      o += 8;
      break;
    default:
      o += deparse_icmp(h.icmp, h.l4 == L4_ICMP6, q + o);
      break;
  }
  if (h.has_vxlan) {
    // Vxlan::deparse (net/src/vxlan/mod.rs:132-145): flags normalized
    q[o] = 0x08; q[o + 1] = q[o + 2] = q[o + 3] = 0;
    q[o + 4] = (h.vni >> 16) & 0xff; q[o + 5] = (h.vni >> 8) & 0xff; q[o + 6] = h.vni & 0xff;
    q[o + 7] = 0;
    o += 8;
  }
  if (h.emb.present) o += deparse_emb(h.emb, q + o);
  return o;
}

// Headers::update_checksums (net/src/headers/mod.rs:894-929)
void update_checksums(Headers &h, const uint8_t *pay, size_t plen) {
  if (h.net == 0) return;
  if (h.net == 4) h.v4.csum = ipv4_checksum(h.v4);
  if (h.has_vxlan) return;
  // the embedded IPv4 header first: it is part of the ICMP payload
  // (headers/mod.rs:906-919; its transport checksum is left as is)
  if (h.emb.present && h.emb.net == 4) h.emb.v4.csum = ipv4_checksum(h.emb.v4);
  Sum16 s;
  switch (h.l4) {
    case L4_NONE: return;
    case L4_UDP: {
      // etherparse UdpHeader::calc_checksum_ipv4/6: pseudo header uses the
      // header's length field; 0 result -> 0xffff
      if (h.net == 4) { s.add_slice(h.v4.src, 4); s.add_slice(h.v4.dst, 4); s.add2(0, 17); s.add_u16(h.udp.len); }
      else { s.add_slice(h.v6.src, 16); s.add_slice(h.v6.dst, 16);
             s.add_u16(0); s.add_u16(h.udp.len); s.add2(0, 0); s.add2(0, 17); }
      s.add_u16(h.udp.sport); s.add_u16(h.udp.dport); s.add_u16(h.udp.len);
      s.add_slice(pay, plen);
      uint16_t c = s.ones_complement();
      h.udp.csum = c == 0 ? 0xffff : c;
      return;
    }
    case L4_TCP: {
      // etherparse TcpHeader::calc_checksum_ipv4/6: tcp_len = header_len + payload
      uint32_t tl = (uint32_t)h.tcp.hlen() + (uint32_t)plen;
      if (h.net == 4) { s.add_slice(h.v4.src, 4); s.add_slice(h.v4.dst, 4); s.add2(0, 6); s.add_u16((uint16_t)tl); }
      else { s.add_slice(h.v6.src, 16); s.add_slice(h.v6.dst, 16);
             s.add_u16((uint16_t)(tl >> 16)); s.add_u16((uint16_t)tl); s.add2(0, 0); s.add2(0, 6); }
      Tcp t = h.tcp;
      t.csum = 0;
      uint8_t tmp[60];
      int n = deparse_tcp(t, tmp);
      s.add_slice(tmp, n);
      s.add_slice(pay, plen);
      h.tcp.csum = s.ones_complement();
      return;
    }
    case L4_ICMP4:
    case L4_ICMP6: {
      if (h.net != (h.l4 == L4_ICMP4 ? 4 : 6)) return;  // debug!("illegal") in the reference
      // an error message with an embedded packet: get_payload_for_checksum
      if (icmp_is_error_msg(h) && h.emb.present) {
        std::vector<uint8_t> v = icmp_checksum_payload(h.emb, pay, plen);
        put16(h.icmp.raw + 2, icmp_checksum(h, v.data(), v.size()));
      } else {
        put16(h.icmp.raw + 2, icmp_checksum(h, pay, plen));
      }
      return;
    }
  }
}

// ---------------------------------------------------------------------------
// Tables
// ---------------------------------------------------------------------------
struct Trie {  // binary trie with LPM (prefix-trie get_lpm semantics)
  struct Node { int32_t child[2]; int64_t val; };
  std::vector<Node> nodes;
  Trie() { nodes.push_back({{-1, -1}, -1}); }
  void insert(const uint8_t *a, int len, int64_t v) {
    int32_t n = 0;
    for (int i = 0; i < len; i++) {
      int b = bit_at(a, i);
      if (nodes[n].child[b] < 0) {
        nodes[n].child[b] = (int32_t)nodes.size();
        nodes.push_back({{-1, -1}, -1});
      }
      n = nodes[n].child[b];
    }
    nodes[n].val = v;  // insert replaces (PrefixMap::insert)
  }
  int64_t lpm(const uint8_t *a, int bits) const {
    int64_t best = nodes[0].val;
    int32_t n = 0;
    for (int i = 0; i < bits; i++) {
      n = nodes[n].child[bit_at(a, i)];
      if (n < 0) break;
      if (nodes[n].val >= 0) best = nodes[n].val;
    }
    return best;
  }
};

// ---------------------------------------------------------------------------
// Masquerade address / port allocator (nat/src/masquerade/apalloc/), with the
// reference's ownership: an allocated port holds its port block, a block its
// address, an address its pool (Arc back-references); dropping the last holder
// releases the tuple (the Drop impls, port_alloc.rs:513-565, alloc.rs:322-326).
// Block i of an address covers ports [256 r, 256 r + 255] for its
// random_index r: i itself (randomize = false), or the shuffle PortAllocator::
// new draws (port_alloc.rs:105-113) -- here the permutation dpgpu.h specifies
// from the configuration's seed and the address (the reference's rand::rng()
// is not reproducible; its draw is replaced by a specified one).  A region's
// offsets are bounded by DP_MASQ_REGION_ADDRS (dpgpu.h), as the reference
// bounds them by u32.
// ---------------------------------------------------------------------------
typedef unsigned __int128 u128;

u128 addr_bits(int fam, const uint8_t *a) {
  u128 v = 0;
  for (int i = 0; i < (fam == 4 ? 4 : 16); i++) v = (v << 8) | a[i];
  return v;
}
Ip bits_addr(int fam, u128 v) {
  Ip r;
  r.fam = (uint8_t)fam;
  const int n = fam == 4 ? 4 : 16;
  for (int i = n - 1; i >= 0; i--) { r.b[i] = (uint8_t)v; v >>= 8; }
  return r;
}
u128 prefix_first(const dp_prefix_t &p) { return addr_bits(p.family, p.addr); }
u128 prefix_last(const dp_prefix_t &p) {
  const int w = p.family == 4 ? 32 : 128;
  const u128 host = p.len >= w ? (u128)0 : (p.len == 0 && w == 128 ? ~(u128)0 : (((u128)1 << (w - p.len)) - 1));
  return prefix_first(p) | host;
}

// AllocatorError (nat/src/masquerade/allocation.rs:12-36)
enum MErr { M_OK = 0, M_NO_FREE_IP, M_NO_PORT_BLOCK, M_NO_FREE_PORT, M_PORT_ALLOC_FAILED,
            M_PORT_RESERVATION_FAILED, M_INTERNAL, M_DENIED, M_NO_POOL_FOUND };
bool m_exhaustion(MErr e) { return e == M_NO_FREE_IP || e == M_NO_PORT_BLOCK || e == M_NO_FREE_PORT; }
// From<&AllocatorError> for DoneReason (allocation.rs:59-73)
int m_done(MErr e) {
  switch (e) {
    case M_NO_FREE_IP: case M_NO_PORT_BLOCK: case M_NO_FREE_PORT: return DP_DONE_NAT_OUT_OF_RESOURCES;
    case M_PORT_ALLOC_FAILED: case M_PORT_RESERVATION_FAILED: return DP_DONE_NAT_FAILURE;
    case M_INTERNAL: return DP_DONE_INTERNAL_FAILURE;
    default: return DP_DONE_FILTERED;  // Denied, NoPoolFound
  }
}

struct MClaim {  // a (prefix, port range) of ReservedPorts (reserved.rs:23)
  dp_prefix_t pfx;
  uint16_t lo, hi;
};

// Bitmap256 (port_alloc.rs:749-882)
struct Bitmap256 {
  uint64_t w[4] = {0, 0, 0, 0};
  bool get(int i) const { return (w[i >> 6] >> (i & 63)) & 1; }
  void set(int i, bool v) { if (v) w[i >> 6] |= 1ull << (i & 63); else w[i >> 6] &= ~(1ull << (i & 63)); }
  bool full() const { return (w[0] & w[1] & w[2] & w[3]) == ~0ull; }
  // Bitmap256::for_block: the claims clipped to the block, port 0 if it may not be given out
  static Bitmap256 for_block(uint16_t base, const std::vector<std::pair<uint16_t, uint16_t>> &claimed,
                             bool reserve_null) {
    Bitmap256 b;
    if (reserve_null && base == 0) b.set(0, true);
    for (auto &r : claimed) {
      const int s = std::max<int>(r.first, base), e = std::min<int>(r.second, base | 0xff);
      for (int p = s; p <= e; p++) b.set(p - base, true);
    }
    return b;
  }
  // allocate_port_from_bitmap: the lowest free offset (trailing ones of each half)
  int alloc() {
    for (int i = 0; i < 256; i++) if (!get(i)) { set(i, true); return i; }
    return -1;
  }
};

struct MPool;
struct MIp;
struct MBlock;

// PortAllocator (port_alloc.rs:84-93); one thread: ThreadPortMap is one slot
struct MPortAlloc {
  bool free[256];
  uint8_t random_index[256];                           // AllocatorPortBlock::random_index
  uint8_t index_of[256];                               // the block with random_index j
  uint16_t usable = 0;
  size_t cur = 0;                                      // current_alloc_index
  int thread_block = -1;
  std::map<size_t, std::weak_ptr<MBlock>> allocated;   // AllocatedPortBlockMap
  std::vector<std::pair<uint16_t, uint16_t>> reserved; // ReservedForAddr
  bool excl_wk = false;
};

// NatPool behind its IpAllocator (alloc.rs:27-30, 336-345)
struct MPool {
  int fam = 4;
  u128 start = 0;
  uint32_t cap = 0;                         // offsets [0, cap)
  std::set<uint32_t> free;                  // PoolBitmap
  std::deque<std::weak_ptr<MIp>> in_use;
  std::vector<MClaim> claims;               // ReservedPorts of the region
  bool excl_wk = false;
  std::shared_ptr<uint32_t> live;           // addresses in use over the allocator (DP_MASQ_ADDRS)
  bool randomize = false;                   // MasqueradeConfig::randomize, and the seed of the shuffles
  uint64_t seed = 0;
};

struct MIp {  // AllocatedIp (alloc.rs:251-255)
  u128 bits = 0;
  uint32_t offset = 0;
  std::shared_ptr<MPool> pool;
  MPortAlloc pa;
  ~MIp() {                                  // Drop: deallocate_from_pool
    pool->free.insert(offset);
    (*pool->live)--;
  }
};

struct MBlock {  // AllocatedPortBlock (port_alloc.rs:396-401)
  std::shared_ptr<MIp> ip;
  uint16_t base = 0;
  size_t index = 0;
  Bitmap256 bm;
  ~MBlock() {  // Drop: deallocate_block (port_alloc.rs:200-212)
    ip->pa.free[index] = true;
    ip->pa.usable++;
  }
};

struct MPort {  // AllocatedPort (port_alloc.rs:530-533)
  uint16_t port = 0;
  bool ident = false;                       // NatPort::Identifier
  std::shared_ptr<MBlock> blk;
  ~MPort() { blk->bm.set(port - blk->base, false); }  // Drop: deallocate_port_from_block
  Ip ip() const { return bits_addr(blk->ip->pool->fam, blk->ip->bits); }
};

// ReservedPorts::for_addr (reserved.rs:45-70): the claims covering the address
std::vector<std::pair<uint16_t, uint16_t>> m_reserved_for(const MPool &P, u128 bits) {
  std::vector<std::pair<uint16_t, uint16_t>> out;
  const Ip a = bits_addr(P.fam, bits);
  for (auto &c : P.claims)
    if (c.pfx.family == P.fam && prefix_covers(c.pfx.addr, c.pfx.len, a.b)) out.push_back({c.lo, c.hi});
  std::sort(out.begin(), out.end());
  return out;
}

// The shuffle of PortAllocator::new as dpgpu.h specifies it: splitmix64 over
// the seed and the address's 32-bit words (most significant first), then
// Fisher-Yates from the last position down
uint64_t m_splitmix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
void m_shuffle_blocks(uint64_t seed, u128 addr, uint8_t out[256]) {
  std::vector<int> base_ports(256);
  for (int i = 0; i < 256; i++) base_ports[i] = i;
  uint64_t x = seed;
  for (int k = 3; k >= 0; k--) x = m_splitmix(x ^ (uint32_t)(addr >> (32 * k)));
  for (int i = 255; i >= 1; i--) {
    x = m_splitmix(x);
    std::swap(base_ports[i], base_ports[x % (uint64_t)(i + 1)]);
  }
  for (int i = 0; i < 256; i++) out[i] = (uint8_t)base_ports[i];
}

// AllocatedIp::new -> PortAllocator::new (port_alloc.rs:100-145)
std::shared_ptr<MIp> m_new_ip(const std::shared_ptr<MPool> &P, uint32_t offset) {
  if (*P->live >= DP_MASQ_ADDRS) return nullptr;
  (*P->live)++;
  auto ip = std::make_shared<MIp>();
  ip->bits = P->start + offset;
  ip->offset = offset;
  ip->pool = P;
  ip->pa.reserved = m_reserved_for(*P, ip->bits);
  ip->pa.excl_wk = P->excl_wk;
  if (P->randomize) m_shuffle_blocks(P->seed, ip->bits, ip->pa.random_index);
  else for (int i = 0; i < 256; i++) ip->pa.random_index[i] = (uint8_t)i;
  for (int i = 0; i < 256; i++) ip->pa.index_of[ip->pa.random_index[i]] = (uint8_t)i;
  for (int i = 0; i < 256; i++) {
    const uint16_t base = (uint16_t)(ip->pa.random_index[i] * 256);
    const bool wk = P->excl_wk && base < 1024;
    const bool whole = Bitmap256::for_block(base, ip->pa.reserved, false).full();
    ip->pa.free[i] = !(wk || whole);
    if (ip->pa.free[i]) ip->pa.usable++;
  }
  return ip;
}

std::shared_ptr<MBlock> m_block_get(MPortAlloc &pa, size_t idx) {  // AllocatedPortBlockMap::get
  auto it = pa.allocated.find(idx);
  if (it == pa.allocated.end()) return nullptr;
  auto b = it->second.lock();
  if (!b) pa.allocated.erase(it);
  return b;
}
bool m_has_free_ports(MPortAlloc &pa) {  // PortAllocator::has_free_ports
  if (pa.usable > 0) return true;
  for (auto &kv : pa.allocated) {
    auto b = kv.second.lock();
    if (b && !b->bm.full()) return true;
  }
  return false;
}
// AllocatedPortBlock::allocate_port_from_block (port_alloc.rs:449-471)
MErr m_port_from_block(const std::shared_ptr<MBlock> &b, bool allow_null, std::shared_ptr<MPort> &out) {
  const int off = b->bm.alloc();
  if (off < 0) return M_NO_FREE_PORT;
  const uint16_t port = (uint16_t)(b->base + off);
  // NatPort::new_port_checked: never 0 (bit 0 of block 0 is preset then)
  if (!allow_null && port == 0) return M_PORT_ALLOC_FAILED;
  auto p = std::make_shared<MPort>();
  p->blk = b;
  p->port = port;
  p->ident = allow_null;
  out = p;
  return M_OK;
}
// PortAllocator::allocate_port (port_alloc.rs:264-284)
MErr m_allocate_port(const std::shared_ptr<MIp> &ip, bool allow_null, std::shared_ptr<MPort> &out) {
  MPortAlloc &pa = ip->pa;
  if (pa.thread_block >= 0) {
    auto cb = m_block_get(pa, (size_t)pa.thread_block);
    if (cb && !cb->bm.full()) return m_port_from_block(cb, allow_null, out);
  }
  // allocate_block: pick_available_block cycling from current_alloc_index
  int idx = -1;
  for (size_t k = 0; k < 256; k++) {
    const size_t i = (pa.cur + k) % 256;
    if (pa.free[i]) { pa.free[i] = false; idx = (int)i; break; }
  }
  if (idx < 0) return M_NO_PORT_BLOCK;
  pa.thread_block = idx;
  pa.cur = (size_t)idx;
  pa.usable--;
  auto b = std::make_shared<MBlock>();
  b->ip = ip;
  b->index = (size_t)idx;
  b->base = (uint16_t)(pa.random_index[idx] * 256);  // AllocatorPortBlock::to_port_number
  b->bm = Bitmap256::for_block(b->base, pa.reserved, !allow_null);
  pa.allocated[(size_t)idx] = b;
  return m_port_from_block(b, allow_null, out);
}
// IpAllocator::allocate (alloc.rs:113-127): cleanup, the addresses in use in
// order, else a new address
MErr m_pool_allocate(const std::shared_ptr<MPool> &P, bool allow_null, std::shared_ptr<MPort> &out) {
  // cleanup_used_ips
  std::deque<std::weak_ptr<MIp>> keep;
  for (auto &w : P->in_use) if (!w.expired()) keep.push_back(w);
  P->in_use.swap(keep);
  // reuse_allocated_ip
  MErr outcome = M_NO_FREE_IP;
  {
    std::vector<std::shared_ptr<MIp>> examined;
    for (auto &w : P->in_use) {
      auto ip = w.lock();
      if (!ip) continue;
      examined.push_back(ip);
      if (!m_has_free_ports(ip->pa)) continue;
      MErr e = m_allocate_port(ip, allow_null, out);
      if (e == M_OK) return M_OK;
      if (e == M_NO_FREE_PORT) continue;
      outcome = e;
      break;
    }
  }
  if (!m_exhaustion(outcome)) return outcome;
  // allocate_from_new_ip: the lowest free offset
  if (P->free.empty()) return M_NO_FREE_IP;
  const uint32_t off = *P->free.begin();
  auto ip = m_new_ip(P, off);
  if (!ip) return M_NO_FREE_IP;  // every address record of the allocator in use
  P->free.erase(P->free.begin());
  P->in_use.push_back(ip);
  return m_allocate_port(ip, allow_null, out);
}

struct MRegion {
  u128 lo, hi;
  std::shared_ptr<MPool> pool;
};
struct MPoolSet {  // PoolSet (alloc.rs:182-185)
  std::vector<MRegion> regions;
  uint64_t idle_ns = 0;
};
// PoolSet::allocate (alloc.rs:208-224)
MErr m_set_allocate(const MPoolSet &S, bool allow_null, std::shared_ptr<MPort> &out) {
  MErr ex = M_OK;
  for (auto &r : S.regions) {
    MErr e = m_pool_allocate(r.pool, allow_null, out);
    if (e == M_OK) return M_OK;
    if (m_exhaustion(e)) { ex = e; continue; }
    return e;
  }
  return ex == M_OK ? M_NO_FREE_IP : ex;
}
// PoolSet::reserve -> IpAllocator::reserve (alloc.rs:140-147, 227-239,
// 437-478) -> PortAllocator::reserve_port (port_alloc.rs:353-374)
MErr m_set_reserve(const MPoolSet &S, const Ip &a, uint16_t port, bool ident, std::shared_ptr<MPort> &out) {
  const u128 bits = addr_bits(a.fam, a.b);
  const MRegion *R = nullptr;
  for (auto &r : S.regions) if (r.lo <= bits && bits <= r.hi) { R = &r; break; }
  if (!R) return M_NO_POOL_FOUND;
  const std::shared_ptr<MPool> &P = R->pool;
  const u128 o = bits - P->start;
  if (o >= P->cap) return M_NO_POOL_FOUND;  // map_address: not an offset this pool serves
  std::shared_ptr<MIp> ip;
  {
    std::vector<std::shared_ptr<MIp>> examined;
    for (auto &w : P->in_use) {
      auto x = w.lock();
      if (!x) continue;
      examined.push_back(x);
      if (x->bits == bits) { ip = x; break; }
    }
  }
  if (!ip) {
    ip = m_new_ip(P, (uint32_t)o);
    if (!ip) return M_NO_POOL_FOUND;
    P->free.erase((uint32_t)o);
    P->in_use.push_back(ip);
  }
  MPortAlloc &pa = ip->pa;
  if (pa.excl_wk && port < 1024) return M_DENIED;
  for (auto &r : pa.reserved) if (r.first <= port && port <= r.second) return M_DENIED;
  // find_block_for_port: the block covering the port, taken if free, else the
  // live block holding it (the retries change nothing single-threaded)
  const size_t idx = pa.index_of[port >> 8];  // try_to_reserve_block: the block that covers it
  std::shared_ptr<MBlock> b;
  if (pa.free[idx]) {
    pa.free[idx] = false;
    pa.usable--;
    b = std::make_shared<MBlock>();
    b->ip = ip;
    b->index = idx;
    b->base = (uint16_t)((port >> 8) * 256);
    b->bm = Bitmap256::for_block(b->base, pa.reserved, !ident);
    pa.allocated[idx] = b;
  } else {
    for (auto &kv : pa.allocated) {
      auto x = kv.second.lock();
      if (x && x->base <= port && port - x->base < 256) { b = x; break; }
    }
    if (!b) return M_PORT_RESERVATION_FAILED;
  }
  if (b->bm.get(port - b->base)) return M_PORT_RESERVATION_FAILED;  // already handed out
  b->bm.set(port - b->base, true);
  auto p = std::make_shared<MPort>();
  p->blk = b;
  p->port = port;
  p->ident = ident;
  out = p;
  return M_OK;
}

// A masquerade expose as the tables hold it (dp_masq_expose_t)
struct MExpose {
  uint32_t src_vni, dst_vni;
  uint64_t idle_ns;
  int fam;
  std::vector<dp_prefix_t> priv, pub;
  std::vector<dp_masq_claim_t> claims;
};

// PoolTableKey (apalloc/mod.rs:111-117) and its table
struct MPoolKey {
  uint8_t proto;
  uint32_t src, dst;
  u128 lo, hi;
  bool operator<(const MPoolKey &o) const {
    if (proto != o.proto) return proto < o.proto;
    if (src != o.src) return src < o.src;
    if (dst != o.dst) return dst < o.dst;
    if (lo != o.lo) return lo < o.lo;
    return hi < o.hi;
  }
};

// NatAllocator (apalloc/mod.rs:248-253)
struct MAlloc {
  std::string config;  // MasqueradeConfig, as its canonical bytes
  uint64_t tag = 0;
  int64_t genid = 0;
  bool randomize = false;
  uint64_t seed = 0;
  std::vector<MExpose> exposes;
  std::map<MPoolKey, MPoolSet> pools[2];  // [0] src44, [1] src66

  // PoolTable::get (apalloc/mod.rs:155-180): of the entries of this protocol
  // and pair of VPCs covering the address, the one starting nearest to it,
  // then the narrowest
  const MPoolSet *lookup(int fam, uint8_t proto, uint32_t src, uint32_t dst, u128 a) const {
    const MPoolSet *best = nullptr;
    u128 bl = 0, bh = 0;
    for (auto &kv : pools[fam == 4 ? 0 : 1]) {
      const MPoolKey &k = kv.first;
      if (k.proto != proto || k.src != src || k.dst != dst || !(k.lo <= a && a <= k.hi)) continue;
      if (!best || k.lo > bl || (k.lo == bl && k.hi < bh)) { best = &kv.second; bl = k.lo; bh = k.hi; }
    }
    return best;
  }
};

// decompose + regions_by_owner (apalloc/region.rs:43-130): the public space
// of the exposes cut into disjoint regions with constant owners; per owner its
// regions, fewest sharers first, then widest, then by address
struct MRegionSpec {
  u128 lo, hi;
  std::vector<size_t> owners;
};
std::vector<MRegionSpec> m_decompose(const std::vector<std::vector<std::pair<u128, u128>>> &own) {
  std::set<u128> cuts;
  for (auto &rs : own)
    for (auto &r : rs) {
      cuts.insert(r.first);
      if (r.second != ~(u128)0) cuts.insert(r.second + 1);
    }
  std::vector<u128> c(cuts.begin(), cuts.end());
  std::vector<MRegionSpec> out;
  for (size_t i = 0; i < c.size(); i++) {
    const u128 s = c[i], e = i + 1 < c.size() ? c[i + 1] - 1 : ~(u128)0;
    std::vector<size_t> owners;
    for (size_t o = 0; o < own.size(); o++)
      for (auto &r : own[o]) if (r.first <= s && s <= r.second) { owners.push_back(o); break; }
    if (owners.empty()) continue;
    if (!out.empty() && out.back().hi + 1 == s && out.back().owners == owners) out.back().hi = e;
    else out.push_back(MRegionSpec{s, e, owners});
  }
  return out;
}

// NatAllocator::new -> build_pools_generic (apalloc/setup.rs:158-204)
std::shared_ptr<MAlloc> m_build(const std::vector<MExpose> &ex, const std::string &cfg, uint64_t tag,
                                int64_t genid, bool randomize, uint64_t seed) {
  auto A = std::make_shared<MAlloc>();
  A->config = cfg;
  A->tag = tag;
  A->genid = genid;
  A->randomize = randomize;
  A->seed = seed;
  A->exposes = ex;
  auto live = std::make_shared<uint32_t>(0);
  for (int fam : {4, 6}) {
    std::map<uint32_t, std::vector<const MExpose *>> groups;  // by destination VPC
    for (auto &e : ex) if (e.fam == fam) groups[e.dst_vni].push_back(&e);
    for (auto &g : groups) {
      for (uint8_t proto : {(uint8_t)6, (uint8_t)17, (uint8_t)(fam == 4 ? 1 : 58)}) {
        std::vector<std::vector<std::pair<u128, u128>>> own;
        for (auto *e : g.second) {
          std::vector<std::pair<u128, u128>> rs;
          for (auto &p : e->pub) rs.push_back({prefix_first(p), prefix_last(p)});
          own.push_back(rs);
        }
        const auto regions = m_decompose(own);
        std::vector<std::shared_ptr<MPool>> pools;
        for (auto &R : regions) {
          auto P = std::make_shared<MPool>();
          P->fam = fam;
          P->start = R.lo;
          const u128 span = R.hi - R.lo;  // len - 1
          P->cap = span >= DP_MASQ_REGION_ADDRS - 1 ? DP_MASQ_REGION_ADDRS : (uint32_t)span + 1;
          for (uint32_t o = 0; o < P->cap; o++) P->free.insert(o);
          P->excl_wk = proto == 6 || proto == 17;
          P->live = live;
          P->randomize = randomize;
          P->seed = seed;
          // claims_for: the claims of every owner, for this protocol (TCP / UDP only)
          const uint32_t bit = proto == 6 ? DP_MASQ_TCP : proto == 17 ? DP_MASQ_UDP : 0;
          for (size_t o : R.owners)
            for (auto &c : g.second[o]->claims)
              if (c.protos & bit) P->claims.push_back(MClaim{c.prefix, c.lo, c.hi});
          pools.push_back(P);
        }
        for (size_t o = 0; o < g.second.size(); o++) {
          std::vector<size_t> mine;
          for (size_t r = 0; r < regions.size(); r++)
            if (std::find(regions[r].owners.begin(), regions[r].owners.end(), o) != regions[r].owners.end())
              mine.push_back(r);
          std::stable_sort(mine.begin(), mine.end(), [&](size_t a, size_t b) {
            const auto &x = regions[a], &y = regions[b];
            if (x.owners.size() != y.owners.size()) return x.owners.size() < y.owners.size();
            const u128 lx = x.hi - x.lo, ly = y.hi - y.lo;
            if (lx != ly) return lx > ly;
            return x.lo < y.lo;
          });
          MPoolSet S;
          S.idle_ns = g.second[o]->idle_ns;
          for (size_t r : mine) S.regions.push_back(MRegion{regions[r].lo, regions[r].hi, pools[r]});
          const MExpose *e = g.second[o];
          for (auto &p : e->priv)  // add_pool_entries: a later expose's entry replaces
            A->pools[fam == 4 ? 0 : 1][MPoolKey{proto, e->src_vni, g.first, prefix_first(p), prefix_last(p)}] = S;
        }
      }
    }
  }
  return A;
}

struct Fib {
  dp_fib_t d;
  Trie v4, v6;
};

struct Rule {
  dp_rule_t r;
  uint32_t orig_index;
};

struct NatEntry {
  dp_nat_entry_t e;
  std::vector<dp_port_range_t> prs;
  std::vector<dp_nat_range_t> ranges;
};
struct NatTable {
  std::vector<NatEntry> entries;
};

// PortFwEntry (nat/src/portfw/portfwtable/objects.rs:30-39) and its id
struct PfRule {
  dp_portfw_rule_t r;
  uint32_t id;
  uint64_t init_ns, estab_ns;  // init_timeout / estab_timeout
};

struct MacKey {
  uint32_t ifindex;
  Ip ip;
  bool operator<(const MacKey &o) const {
    if (ifindex != o.ifindex) return ifindex < o.ifindex;
    if (ip.fam != o.ip.fam) return ip.fam < o.ip.fam;
    return memcmp(ip.b, o.ip.b, 16) < 0;
  }
};

}  // namespace

struct dpo_tables {
  int64_t genid = 0;
  std::vector<Fib> fibs;
  std::unordered_map<uint32_t, uint32_t> vni_fib;  // vni -> fib index
  std::unordered_map<uint32_t, uint32_t> vrf_fib;  // vrf id -> fib index
  std::vector<dp_route_nh_t> nhs;
  std::vector<dp_fib_entry_t> entries;
  std::vector<dp_instr_t> instrs;
  std::unordered_map<uint32_t, dp_iface_t> ifaces;
  std::map<MacKey, dp_adjacency_t> adjs;
  std::vector<Rule> acl4, acl6;
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> acl_default;
  std::vector<Rule> ffr4, ffl4, ffr6, ffl6;
  std::map<uint32_t, NatTable> nat_dst;                          // src_vni
  std::map<std::pair<uint32_t, uint32_t>, NatTable> nat_src;     // (src_vni, dst_vni)
  std::vector<PfRule> pf;   // PortFwTable entries (ids stable across generations)
  uint32_t pf_next_id = 1;  // the lineage's next entry id
  // MasqueradeConfig: the masquerade exposes, their canonical bytes, the tag
  std::vector<MExpose> masq;
  std::string masq_cfg;
  uint64_t masq_tag = 0;
  bool masq_random = false;  // MasqueradeConfig::randomize and the shuffles' seed
  uint64_t masq_seed = 0;
  uint64_t serial = 0;      // this build (a flow table syncs its allocator once per build)
};

namespace {
// FlowInfo (net/src/flows/flow_info.rs:189-199) without masquerade state;
// `related` is the Weak of related_pair, alive while the related flow is in
// the table.  The port-forwarding state (PortFwState, nat/src/portfw/
// flow_state.rs:29-35): action, use_ip / use_port, the rule's Weak (an entry
// id, alive while the tables hold that entry) and the NatFlowStatus shared
// with the related flow (an index into dpo_flows::nfs).
struct OFlow {
  dp_flow_t d{};
  FKey key;
  uint32_t status = DP_FLOW_DETACHED;
  int64_t related = -1;
  bool in_table = false;
  uint8_t pf = DP_PF_NONE;
  int64_t pf_status = -1;
  Ip pf_ip;
  uint16_t pf_port = 0;
  uint32_t pf_rule = 0;
  // MasqueradeState (nat/src/masquerade/state.rs:13-20): action, use_ip /
  // use_port (NatPort: a port, or an ICMP identifier), idle timeout, the
  // NatFlowStatus cell shared with the related flow, and the allocation the
  // SrcNat flow owns
  uint8_t masq = DP_PF_NONE;
  int64_t m_status = -1;
  Ip m_ip;
  uint16_t m_port = 0;
  bool m_ident = false;
  uint64_t m_idle_ns = 0;
  std::shared_ptr<MPort> m_alloc;
};
}  // namespace

// FlowTable (flow-entry/src/flow_table/table.rs:24-330)
struct dpo_flows {
  std::vector<OFlow> f;                                 // every FlowInfo ever made (ref = index)
  std::unordered_map<FKey, uint64_t, FKeyHash> map;     // the table
  uint64_t capacity = 10000000;                         // FlowTable::DEFAULT_CAPACITY
  std::vector<uint8_t> nfs;                             // AtomicNatFlowStatus cells
  uint64_t now = 0;                                     // Instant::now() (ns, DP_OPT_CLOCK)
  // NatAllocatorWriter's slot (nat/src/masquerade/allocator_writer.rs:95):
  // the allocator masquerade flows of this table draw from, and the tables
  // build it reflects
  std::shared_ptr<MAlloc> alloc;
  uint64_t synced = 0;
  // flows that left the table during the running burst: their allocations are
  // released when the burst ends (a detached FlowInfo lives on in its timer
  // task until the runtime polls it, table.rs:161-213)
  bool in_burst = false;
  std::vector<int64_t> departed;
};

namespace {

// ---------------------------------------------------------------------------
// Classifier: first match over rules in match order
// (acl/src/reference/table.rs:94-101; predicates match-action/src/predicate.rs)
// ---------------------------------------------------------------------------
struct Key {
  uint8_t proto;
  uint32_t a, b;
  uint8_t gate;
  const uint8_t *src, *dst;
  uint16_t sport, dport;
};

bool rule_matches(const dp_rule_t &r, const Key &k, int fam) {
  if ((k.proto & r.proto_mask) != (r.proto_val & r.proto_mask)) return false;
  if (k.a != r.vni_a || k.b != r.vni_b || k.gate != r.gate) return false;
  (void)fam;
  if (!prefix_covers(r.src.addr, r.src.len, k.src)) return false;
  if (!prefix_covers(r.dst.addr, r.dst.len, k.dst)) return false;
  if (k.sport < r.sport_lo || k.sport > r.sport_hi) return false;
  if (k.dport < r.dport_lo || k.dport > r.dport_hi) return false;
  return true;
}

int64_t classify(const std::vector<Rule> &rules, const Key &k, int fam) {
  for (size_t i = 0; i < rules.size(); i++)
    if (rule_matches(rules[i].r, k, fam)) return (int64_t)i;
  return -1;
}

// ---------------------------------------------------------------------------
// Static NAT lookups (nat/src/static_nat/setup/tables.rs:94-209,
// lpm/src/trie/ip_port_prefix_trie.rs:80-97, lpm/src/prefix/range_map.rs:68-81)
// ---------------------------------------------------------------------------
bool covers_port(const NatEntry &e, uint16_t port) {
  if (!e.e.is_pat) return true;
  for (auto &pr : e.prs) if (pr.lo <= port && port <= pr.hi) return true;
  return false;
}
bool covers_all_ports(const NatEntry &e) {
  if (!e.e.is_pat) return true;
  uint64_t sum = 0;
  for (auto &pr : e.prs) sum += (uint64_t)pr.hi - pr.lo + 1;
  return sum == 65536;
}

// returns 1 and new addr (+ port, has_new_port) or 0
int nat_find_mapping(const NatTable &t, const uint8_t *addr, bool has_port, uint16_t port,
                     uint32_t &new_addr, bool &has_new_port, uint16_t &new_port) {
  // IpPortPrefixTrie::lookup: matching prefixes, longest first
  std::vector<const NatEntry *> match;
  for (auto &e : t.entries)
    if (e.e.prefix.family == 4 && prefix_covers(e.e.prefix.addr, e.e.prefix.len, addr))
      match.push_back(&e);
  std::stable_sort(match.begin(), match.end(), [](const NatEntry *x, const NatEntry *y) {
    return x->e.prefix.len > y->e.prefix.len;
  });
  const NatEntry *hit = nullptr;
  for (auto *e : match) {
    if (has_port && covers_port(*e, port)) { hit = e; break; }
    if (covers_all_ports(*e)) { hit = e; break; }
  }
  if (!hit) return 0;
  uint32_t a = be32(addr);
  uint32_t net = be32(hit->e.prefix.addr);
  uint64_t ip_off = (uint64_t)(a - net);
  if (!hit->e.is_pat) {
    // AddrTranslationValue::get_entry
    uint64_t entry_offset = ip_off;
    if (entry_offset >= hit->e.size) return 0;
    // ranges_tree.lookup(addr): greatest key start <= addr, then addr <= end
    const dp_nat_range_t *rg = nullptr;
    for (auto &r : hit->ranges)
      if (be32(r.orig_lo_ip) <= a) rg = &r;  // sorted ascending
    if (!rg || a > be32(rg->orig_hi_ip)) return 0;
    uint64_t o2 = entry_offset - rg->offset;
    uint64_t tlen = (uint64_t)be32(rg->tgt_hi_ip) - be32(rg->tgt_lo_ip) + 1;
    if (o2 >= tlen) return 0;
    new_addr = (uint32_t)(be32(rg->tgt_lo_ip) + o2);
    has_new_port = false;
    return 1;
  }
  // PAT: a port is required
  if (!has_port) return 0;
  const dp_port_range_t *ppr = nullptr;
  for (auto &pr : hit->prs) if (pr.lo <= port && port <= pr.hi) { ppr = &pr; break; }
  if (!ppr) return 0;  // unreachable in the reference
  uint64_t plen = (uint64_t)ppr->hi - ppr->lo + 1;
  uint64_t entry_offset = ip_off * plen + (uint64_t)(port - ppr->lo);
  if (entry_offset >= hit->e.size) return 0;
  // ranges_tree.lookup(IpPort): lexicographic (ip, port)
  const dp_nat_range_t *rg = nullptr;
  for (auto &r : hit->ranges) {
    uint32_t lo = be32(r.orig_lo_ip);
    if (lo < a || (lo == a && r.orig_lo_port <= port)) rg = &r;
  }
  if (!rg) return 0;
  uint32_t hi = be32(rg->orig_hi_ip);
  if (a > hi || (a == hi && port > rg->orig_hi_port)) return 0;
  uint64_t o2 = entry_offset - rg->offset;
  uint64_t tpl = (uint64_t)rg->tgt_hi_port - rg->tgt_lo_port + 1;
  uint64_t tip = (uint64_t)be32(rg->tgt_hi_ip) - be32(rg->tgt_lo_ip) + 1;
  if (o2 >= tip * tpl) return 0;
  uint64_t io = o2 / tpl, po = o2 % tpl;
  new_addr = (uint32_t)(be32(rg->tgt_lo_ip) + io);
  new_port = (uint16_t)(rg->tgt_lo_port + po);
  if (new_port == 0) return 0;  // "Found port 0 ... cannot use it for PAT"
  has_new_port = true;
  return 1;
}

// ---------------------------------------------------------------------------
// Pipeline stages
// ---------------------------------------------------------------------------
const dp_iface_t *find_iface(const dpo_tables &T, uint32_t ifindex) {
  auto it = T.ifaces.find(ifindex);
  return it == T.ifaces.end() ? nullptr : &it->second;
}

bool iface_has_mac(const dp_iface_t &i) {
  return i.iftype == DP_IFT_ETHERNET || i.iftype == DP_IFT_DOT1Q;
}

// Ingress (dataplane/src/packet_processor/ingress.rs:153-182)
void stage_ingress(const dpo_tables &T, Packet &p, uint32_t iif) {
  if (p.is_done()) return;
  const dp_iface_t *i = find_iface(T, iif);
  if (!i) { p.done(DP_DONE_INTERFACE_UNKNOWN); return; }
  if (i->admin_state == DP_IF_DOWN) { p.done(DP_DONE_INTERFACE_ADM_DOWN); return; }
  if (!iface_has_mac(*i)) { p.done(DP_DONE_INTERFACE_UNSUPPORTED); return; }
  if (!p.h.has_eth) { p.done(DP_DONE_NOT_ETHERNET); return; }
  static const uint8_t bcast[6] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
  if (memcmp(p.h.eth.dst, bcast, 6) == 0) {
    p.m.flags |= DP_META_IS_L2_BCAST;
    p.done(DP_DONE_UNHANDLED);
  } else if (memcmp(p.h.eth.dst, i->mac, 6) == 0) {
    switch (i->attach) {
      case DP_ATTACH_VRF:
        if (p.h.net == 0) { p.done(DP_DONE_NOT_IP); return; }
        p.m.has_vrf = true;
        p.m.vrf = i->vrf_id;
        break;
      case DP_ATTACH_BRIDGE: p.done(DP_DONE_INTERFACE_UNSUPPORTED); break;
      default: p.done(DP_DONE_INTERFACE_DETACHED); break;
    }
  } else {
    p.done(DP_DONE_MAC_NOT_FOR_US);
  }
}

Ip ip_dst(const Headers &h) { return h.net == 4 ? ip4(h.v4.dst) : ip6(h.v6.dst); }

// The bytes the Hasher calls of net/src/packet/hash.rs:17-68 feed it, in
// order, under the Hasher trait's default encodings: write_uN(v) = v's
// native (little-endian) bytes, a slice's length prefix = write_usize.
// Field types: Ipv4Addr / Ipv6Addr hash as write_u32 / write_u128
// of from_ne_bytes(octets) (the octets in order), IpNumber write_u8, ports,
// VIDs, ethertypes and ICMP identifiers write_u16, MACs ([u8; 6]) a length
// prefix and six bytes.
void hash_u16(std::vector<uint8_t> &o, uint16_t v) { o.push_back((uint8_t)v); o.push_back((uint8_t)(v >> 8)); }
void hash_usize(std::vector<uint8_t> &o, uint64_t v) { for (int i = 0; i < 8; i++) o.push_back((uint8_t)(v >> (8 * i))); }
void hash_ip_bytes(const Headers &h, std::vector<uint8_t> &o) {  // hash_ip (hash.rs:17-54)
  if (h.net == 0) return;
  if (h.net == 4) { o.insert(o.end(), h.v4.src, h.v4.src + 4); o.insert(o.end(), h.v4.dst, h.v4.dst + 4); o.push_back(h.v4.proto); }
  else { o.insert(o.end(), h.v6.src, h.v6.src + 16); o.insert(o.end(), h.v6.dst, h.v6.dst + 16); o.push_back(h.v6.nh); }
  if (h.l4 == L4_TCP) { hash_u16(o, h.tcp.sport); hash_u16(o, h.tcp.dport); }
  else if (h.l4 == L4_UDP) { hash_u16(o, h.udp.sport); hash_u16(o, h.udp.dport); }
  else if ((h.l4 == L4_ICMP4 && (h.icmp.raw[0] == 0 || h.icmp.raw[0] == 8)) ||
           (h.l4 == L4_ICMP6 && (h.icmp.raw[0] == 128 || h.icmp.raw[0] == 129)))
    hash_u16(o, (uint16_t)((h.icmp.raw[4] << 8) | h.icmp.raw[5]));
}

// packet_hash_ecmp (net/src/packet/hash.rs:74-78)
uint64_t hash_ecmp(const Headers &h) {
  std::vector<uint8_t> o;
  hash_ip_bytes(h, o);
  return rapid(o.data(), o.size());
}
// packet_hash_vxlan (net/src/packet/hash.rs:84-88)
uint16_t hash_vxlan(const Headers &h) {
  std::vector<uint8_t> o;
  if (h.has_eth) {  // hash_l2_frame (hash.rs:57-68)
    hash_usize(o, 6);
    o.insert(o.end(), h.eth.src, h.eth.src + 6);
    hash_usize(o, 6);
    o.insert(o.end(), h.eth.dst, h.eth.dst + 6);
    hash_u16(o, h.eth.type);
  }
  for (auto &v : h.vlans) hash_u16(o, v.vid());
  hash_ip_bytes(h, o);
  uint64_t x = rapid(o.data(), o.size());
  return (uint16_t)(x % 16384 + 49152);
}

int64_t fib_lpm(const Fib &f, const Ip &a) {
  return a.fam == 4 ? f.v4.lpm(a.b, 32) : f.v6.lpm(a.b, 128);
}

// Packet::vxlan_decap (net/src/packet/mod.rs:227-259)
// returns 1 ok, 0 not vxlan, -1 inner parse error
int vxlan_decap(Packet &p, uint32_t &vni) {
  if (!p.h.has_vxlan) return 0;
  bool has_q = p.h.net != 0;
  uint8_t dscp = 0, ecn = 0;
  if (p.h.net == 4) { dscp = p.h.v4.dscp; ecn = p.h.v4.ecn; }
  if (p.h.net == 6) { dscp = p.h.v6.tc >> 2; ecn = p.h.v6.tc & 3; }
  Headers inner;
  int c = parse_headers(p.buf + p.pay_start, p.pay_end - p.pay_start, inner);
  if (c < 0) return -1;
  vni = p.h.vni;
  p.pay_start += (uint64_t)c;
  p.h = inner;
  if (has_q) { p.m.has_dscp = true; p.m.dscp = dscp; p.m.ecn = ecn; }
  return 1;
}

void ipf_decrement_ttl(Packet &p) {  // ipforward.rs:369-390
  if (p.h.net == 4) {
    if (p.h.v4.ttl == 0) { p.done(DP_DONE_HOP_LIMIT_EXCEEDED); return; }
    p.h.v4.ttl--;
    if (p.h.v4.ttl == 0) p.done(DP_DONE_HOP_LIMIT_EXCEEDED);
  } else {
    if (p.h.v6.hop == 0) { p.done(DP_DONE_HOP_LIMIT_EXCEEDED); return; }
    p.h.v6.hop--;
    if (p.h.v6.hop == 0) p.done(DP_DONE_HOP_LIMIT_EXCEEDED);
  }
}

// IpForwarder::vxlan_encap (ipforward.rs:222-289) + Packet::vxlan_encap
// (net/src/packet/mod.rs:279-326) + build_vxlan_headers (ipforward.rs:181-219)
void ipf_vxlan_encap(const dpo_tables &T, Packet &p, const dp_instr_t &in, const Fib &f) {
  if (!(f.d.flags & DP_FIB_VTEP_HAS_MAC)) { p.done(DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  if (!(in.flags & DP_INSTR_HAS_DMAC)) { p.done(DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  static const uint8_t zero[6] = {0};
  // set_eth_source: SourceMac::new (non-zero, unicast); no-op without Eth
  if (memcmp(f.d.vtep_mac, zero, 6) == 0 || (f.d.vtep_mac[0] & 1)) { p.done(DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  if (p.h.has_eth) memcpy(p.h.eth.src, f.d.vtep_mac, 6);
  // set_eth_destination: DestinationMac::new (non-zero)
  if (memcmp(in.mac, zero, 6) == 0) { p.done(DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  if (p.h.has_eth) memcpy(p.h.eth.dst, in.mac, 6);
  if (p.m.flags & DP_META_REFR_CHKSUM) {
    update_checksums(p.h, p.buf + p.pay_start, p.pay_end - p.pay_start);
    p.m.flags &= ~DP_META_REFR_CHKSUM;
  } else if (p.h.net == 4) {
    p.h.v4.csum = ipv4_checksum(p.h.v4);
  } else {
    // `unreachable!()` in the reference (non-IPv4 without refresh): panic.
    p.done(DP_DONE_INTERNAL_FAILURE);
    return;
  }
  // build_vxlan_headers
  if (!(f.d.flags & DP_FIB_VTEP_HAS_IP)) { p.done(DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  const dp_ipaddr_t &sip = f.d.vtep_ip;
  const dp_ipaddr_t &dip = in.addr;
  Headers outer;
  if (sip.family == 4 && dip.family == 4) {
    if ((sip.addr[0] & 0xf0) == 0xe0 || (sip.addr[0] == 255 && sip.addr[1] == 255 && sip.addr[2] == 255 && sip.addr[3] == 255)) {
      p.done(DP_DONE_VXLAN_ENCAP_FAILURE); return;
    }
    outer.net = 4;
    Ipv4 &o = outer.v4;
    memset(&o, 0, sizeof(o));
    // etherparse Ipv4Header::default(): DF set, id 0, ttl 0, proto 255
    // (assumption; DESIGN.md "unpinned"); then src/dst/ttl 64/proto UDP
    o.df = true;
    memcpy(o.src, sip.addr, 4);
    memcpy(o.dst, dip.addr, 4);
    o.ttl = 64;
    o.proto = 17;
  } else if (sip.family == 6 && dip.family == 6) {
    if (sip.addr[0] == 0xff) { p.done(DP_DONE_VXLAN_ENCAP_FAILURE); return; }
    outer.net = 6;
    Ipv6 &o = outer.v6;
    memset(&o, 0, sizeof(o));
    memcpy(o.src, sip.addr, 16);
    memcpy(o.dst, dip.addr, 16);
    o.hop = 64;
    o.nh = 17;
  } else {
    p.done(DP_DONE_VXLAN_ENCAP_FAILURE);
    return;
  }
  // Packet::vxlan_encap: deparse inner headers into the payload front
  int need = p.h.size();
  if ((int64_t)p.pay_start - need < (int64_t)p.room_start) {
    p.done(DP_DONE_VXLAN_ENCAP_FAILURE);  // Prepend error
    return;
  }
  uint16_t sport = hash_vxlan(p.h);
  deparse_headers(p.h, p.buf + p.pay_start - need);
  p.pay_start -= (uint64_t)need;
  uint64_t len = (p.pay_end - p.pay_start) + 16;
  outer.l4 = L4_UDP;
  outer.udp.sport = sport;
  outer.udp.dport = 4789;
  outer.udp.len = (uint16_t)len;
  outer.udp.csum = 0;
  outer.has_vxlan = true;
  outer.vni = in.vni;
  // apply_outer_qos_to_ip_headers (net/src/packet/mod.rs:163-188)
  if (outer.net == 4) {
    if (p.m.has_dscp) { outer.v4.dscp = p.m.dscp; outer.v4.ecn = p.m.ecn; }
    outer.v4.total_len = (uint16_t)(outer.v4.hlen() + len);
    outer.v4.csum = ipv4_checksum(outer.v4);
  } else {
    if (p.m.has_dscp) outer.v6.tc = (uint8_t)((p.m.dscp << 2) | p.m.ecn);
    outer.v6.plen = (uint16_t)len;
  }
  p.h = outer;  // no Eth: Egress adds it
  p.m.dst_vni = in.vni;
}

void ipf_exec(const dpo_tables &T, Packet &p, const dp_instr_t &in, const Fib &f) {
  switch (in.kind) {
    case DP_INSTR_DROP: p.done(DP_DONE_ROUTE_DROP); break;
    case DP_INSTR_LOCAL: {
      uint32_t vni = 0;
      int r = vxlan_decap(p, vni);
      if (r == 0) { p.done(DP_DONE_LOCAL); break; }
      if (r < 0) { p.done(DP_DONE_VXLAN_DECAP_FAILURE); break; }
      auto it = T.vni_fib.find(vni);
      if (it == T.vni_fib.end()) { p.done(DP_DONE_UNROUTABLE); break; }
      p.m.src_vni = vni;
      p.m.has_vrf = true;
      p.m.vrf = T.fibs[it->second].d.vrf_id;
      p.m.flags |= DP_META_IS_OVERLAY;
      break;
    }
    case DP_INSTR_ENCAP_VXLAN: ipf_vxlan_encap(T, p, in, f); break;
    case DP_INSTR_EGRESS:
      p.m.has_oif = in.flags & DP_INSTR_HAS_IFINDEX;
      p.m.oif = in.ifindex;
      p.m.has_nh = in.flags & DP_INSTR_HAS_ADDR;
      if (p.m.has_nh) { p.m.nh.fam = in.addr.family; memcpy(p.m.nh.b, in.addr.addr, 16); }
      break;
  }
}

// IpForwarder::forward_packet (ipforward.rs:54-121)
void stage_ipforward(const dpo_tables &T, Packet &p) {
  if (p.is_done()) return;
  bool had_vrf = p.m.has_vrf;
  uint32_t vrf0 = p.m.vrf;
  const Fib *f = nullptr;
  if (p.m.dst_vni) {
    auto it = T.vni_fib.find(p.m.dst_vni);
    if (p.h.net == 0) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
    if (it == T.vni_fib.end()) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
    f = &T.fibs[it->second];
  } else if (p.m.has_vrf) {
    auto it = T.vrf_fib.find(p.m.vrf);
    if (p.h.net == 0) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
    if (it == T.vrf_fib.end()) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
    f = &T.fibs[it->second];
  } else {
    if (p.overlay()) p.done(DP_DONE_INTERNAL_FAILURE);
    return;
  }
  Ip dst = ip_dst(p.h);
  int64_t nhi = fib_lpm(*f, dst);
  if (nhi < 0) { p.done(DP_DONE_INTERNAL_FAILURE); return; }  // a /0 always exists
  const dp_route_nh_t &nh = T.nhs[nhi];
  uint32_t idx = 0;
  if (nh.n_entries > 1) idx = (uint32_t)(hash_ecmp(p.h) % nh.n_entries);
  uint32_t ei = nh.first_entry + idx;
  const dp_fib_entry_t &e = T.entries[ei];
  p.m.fib_entry = ei;
  bool iplocal = e.n_instr == 1 && T.instrs[e.first_instr].kind == DP_INSTR_LOCAL;
  if (!iplocal) {
    ipf_decrement_ttl(p);
    if (p.is_done()) return;
  }
  for (uint32_t k = 0; k < e.n_instr; k++) {
    ipf_exec(T, p, T.instrs[e.first_instr + k], *f);
    if (p.is_done()) return;
  }
  if (p.m.has_vrf == had_vrf && (!had_vrf || p.m.vrf == vrf0)) p.m.has_vrf = false;
}

// --- flow table ----------------------------------------------------------
void flow_invalidate(dpo_flows *FL, int64_t r) {  // FlowInfo::invalidate (flow_info.rs:435-442)
  if (FL && r >= 0) FL->f[r].status = DP_FLOW_CANCELLED;
}
bool flow_alive(const dpo_flows *FL, int64_t r) { return r >= 0 && FL->f[r].in_table; }
// A flow left the table: its FlowInfo (and the allocation its masquerade
// state owns) is dropped now, or when the running burst ends.
void flow_depart(dpo_flows *FL, int64_t r) {
  if (FL->in_burst) FL->departed.push_back(r);
  else FL->f[r].m_alloc.reset();
}
void flow_invalidate_pair(dpo_flows *FL, int64_t r) {  // invalidate_pair (flow_info.rs:449-455)
  if (!FL || r < 0) return;
  flow_invalidate(FL, r);
  if (flow_alive(FL, FL->f[r].related)) flow_invalidate(FL, FL->f[r].related);
}
int64_t flow_find(const dpo_flows *FL, const FKey &k) {  // FlowTable::lookup (table.rs:267-275)
  auto it = FL->map.find(k);
  return it == FL->map.end() ? -1 : (int64_t)it->second;
}
void key_addrs(FKey &k, int fam, const uint8_t *src, const uint8_t *dst) {
  k.fam = (uint8_t)fam;
  memcpy(k.src, src, fam == 4 ? 4 : 16);
  memcpy(k.dst, dst, fam == 4 ? 4 : 16);
}
// FlowKey::try_from(&Packet) (flow_key.rs:589-621).  false: no key, or an
// ICMP error key (IcmpProtoKey::ErrorMsgData), which no flow ever has.
bool packet_flow_key(const Packet &p, FKey &k) {
  if (p.h.net == 0) return false;
  k = FKey{};
  k.vni = p.m.src_vni;
  if (p.h.net == 4) key_addrs(k, 4, p.h.v4.src, p.h.v4.dst);
  else key_addrs(k, 6, p.h.v6.src, p.h.v6.dst);
  switch (p.h.l4) {
    case L4_TCP: k.kind = DP_FLOW_TCP; k.sp = p.h.tcp.sport; k.dp = p.h.tcp.dport; return true;
    case L4_UDP: k.kind = DP_FLOW_UDP; k.sp = p.h.udp.sport; k.dp = p.h.udp.dport; return true;
    case L4_ICMP4:
    case L4_ICMP6: {
      // IcmpProtoKey::new_icmp_v4/v6 (flow_key.rs:318-338): Echo Request /
      // Reply (etherparse decodes them with code 0) carry their identifier
      const bool v6 = p.h.l4 == L4_ICMP6;
      const uint8_t t = p.h.icmp.raw[0], c = p.h.icmp.raw[1];
      const bool echo = c == 0 && (v6 ? (t == 128 || t == 129) : (t == 0 || t == 8));
      if (echo) { k.kind = DP_FLOW_ICMP_QUERY; k.sp = be16(p.h.icmp.raw + 4); return true; }
      if (icmp_is_error_msg(p.h)) return false;
      k.kind = DP_FLOW_ICMP_OTHER;
      return true;
    }
    default: return false;
  }
}
// FlowLookup::process (flow-entry/src/flow_table/nf_lookup.rs:34-55)
void stage_flow_lookup(const dpo_flows *FL, Packet &p) {
  if (!FL || p.is_done() || !p.overlay() || p.m.dst_vni) return;
  FKey k;
  if (packet_flow_key(p, k)) p.flow = flow_find(FL, k);
}
// FlowSummary::from_meta (flow-filter/src/lib.rs:380-398): every stored flow
// has a destination VPC and no masquerade state.
struct FlowSummary {
  bool present = false;
  int64_t genid = 0;
  uint32_t dst_vni = 0;
  bool needs_pf = false;
  bool needs_masq = false;
};

// FlowFilter (flow-filter/src/lib.rs:75-246, context/tables.rs:800-915), in
// the reference's burst phases: classify + lookup (A, B) for every packet of
// the burst, then apply_route (C) for every packet.
struct FfWork {
  bool lookup = false;
  uint8_t gate = 0;  // SourceGate of the local lookup (1: PortFwdReply)
  uint32_t gate_vni = 0;  // LookupInput.dst_vpcd: the GateVni of the remote lookup
  FlowSummary fs;
  int64_t ri = -1, li = -1;  // remote / local rule (-1: miss)
};
void ff_classify(const dpo_tables &T, const dpo_flows *FL, Packet &p, FfWork &w) {
  w = FfWork{};
  if (p.is_done() || !p.overlay() || p.m.dst_vni) return;
  if (FL && p.flow >= 0) {
    const OFlow &f = FL->f[p.flow];
    w.fs = FlowSummary{true, f.d.genid, f.d.dst_vni, f.pf != DP_PF_NONE, f.masq != DP_PF_NONE};
    // dst_vpcd_from_valid_flow (lib.rs:327-349) -> tag_for_bypass (:213-231)
    if (f.status == DP_FLOW_ACTIVE && f.d.genid >= T.genid) {
      p.m.dst_vni = f.d.dst_vni;
      if (w.fs.needs_masq) p.m.flags |= DP_META_REQ_MASQUERADE;
      if (w.fs.needs_pf) p.m.flags |= DP_META_REQ_PORT_FORWARDING;
      if (f.d.flags & DP_FLOW_REQ_STATIC_NAT_SRC) p.m.flags |= DP_META_REQ_STATIC_NAT_SRC;
      if (f.d.flags & DP_FLOW_REQ_STATIC_NAT_DST) p.m.flags |= DP_META_REQ_STATIC_NAT_DST;
      return;
    }
    // flow_revalidation_data (:296-325): the reply flow of a masqueraded
    // pair is revalidated against the remote rules gated on its destination
    // VPC, that of a port-forwarded pair against the local rules gated on
    // PortFwdReply
    if (f.status == DP_FLOW_ACTIVE && f.d.genid < T.genid && !(f.d.flags & DP_FLOW_INITIATOR)) {
      if (w.fs.needs_masq) w.gate_vni = f.d.dst_vni;
      else if (w.fs.needs_pf) w.gate = 1;
    }
  }
  if (p.h.net == 0) { p.done(DP_DONE_NOT_IP); return; }
  if (!p.m.src_vni) { p.done(DP_DONE_UNROUTABLE); return; }
  w.lookup = true;
  uint8_t proto = p.h.net == 4 ? p.h.v4.proto : p.h.v6.nh;
  uint16_t sp = 0, dpp = 0;
  if (p.h.l4 == L4_TCP) { sp = p.h.tcp.sport; dpp = p.h.tcp.dport; }
  if (p.h.l4 == L4_UDP) { sp = p.h.udp.sport; dpp = p.h.udp.dport; }
  const uint8_t *src = p.h.net == 4 ? p.h.v4.src : p.h.v6.src;
  const uint8_t *dst = p.h.net == 4 ? p.h.v4.dst : p.h.v6.dst;
  const auto &rem = p.h.net == 4 ? T.ffr4 : T.ffr6;
  const auto &loc = p.h.net == 4 ? T.ffl4 : T.ffl6;
  static const uint8_t zero16[16] = {0};
  Key k{proto, p.m.src_vni, w.gate_vni /* GateVni: 0 = dst_vpcd None */, 0, zero16, dst, 0, dpp};
  w.ri = classify(rem, k, p.h.net);
  if (w.ri < 0) return;  // DestinationMiss
  Key k2{proto, p.m.src_vni, rem[w.ri].r.action, w.gate, src, zero16, sp, 0};
  w.li = classify(loc, k2, p.h.net);
}
void ff_apply(const dpo_tables &T, dpo_flows *FL, Packet &p, const FfWork &w) {
  if (!w.lookup) return;
  if (w.ri < 0 || w.li < 0) {  // DestinationMiss / SourceMiss (lib.rs:174-185)
    flow_invalidate_pair(FL, p.flow);
    p.done(DP_DONE_FILTERED);
    return;
  }
  const auto &rem = p.h.net == 4 ? T.ffr4 : T.ffr6;
  const auto &loc = p.h.net == 4 ? T.ffl4 : T.ffl6;
  const dp_rule_t &rv = rem[w.ri].r;
  uint32_t src_nat = loc[w.li].r.action, dst_nat = rv.action2;
  p.m.dst_vni = rv.action;
  // set_nat_requirements (flow-filter/src/lib.rs:233-246)
  auto apply = [&](uint32_t mode, uint32_t stat_flag) {
    if (mode == DP_NAT_MASQUERADE) p.m.flags |= DP_META_REQ_MASQUERADE;
    if (mode == DP_NAT_STATIC) p.m.flags |= stat_flag;
    if (mode == DP_NAT_PORT_FORWARDING) p.m.flags |= DP_META_REQ_PORT_FORWARDING;
  };
  apply(src_nat, DP_META_REQ_STATIC_NAT_SRC);
  apply(dst_nat, DP_META_REQ_STATIC_NAT_DST);
  // the key before static NAT, for the flows port forwarding / masquerade
  // create (lib.rs:193-201)
  const uint32_t stat = DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST;
  if ((p.m.flags & (DP_META_REQ_PORT_FORWARDING | DP_META_REQ_MASQUERADE)) && (p.m.flags & stat))
    p.has_ikey = packet_flow_key(p, p.ikey);
  // should_invalidate_flow (lib.rs:258-294): a flow of another generation is
  // outdated if its destination or its NAT requirements differ, or if none
  // of its stateful NAT is still required
  if (w.fs.present && w.fs.genid != T.genid) {
    const bool pf = p.m.flags & DP_META_REQ_PORT_FORWARDING, masq = p.m.flags & DP_META_REQ_MASQUERADE;
    if (w.fs.dst_vni != p.m.dst_vni || masq != w.fs.needs_masq || pf != w.fs.needs_pf || (!pf && !masq))
      flow_invalidate_pair(FL, p.flow);
  }
}

// AclFilter (acl-filter/src/lib.rs:51-152)
void stage_acl(const dpo_tables &T, dpo_flows *FL, Packet &p) {
  if (p.is_done() || !p.overlay()) return;
  if (!p.m.src_vni || !p.m.dst_vni) { p.done(DP_DONE_UNROUTABLE); return; }
  if (p.h.net == 0) { p.done(DP_DONE_NOT_IP); return; }
  uint8_t proto = p.h.net == 4 ? p.h.v4.proto : p.h.v6.nh;
  uint16_t sp = 0, dpp = 0;
  if (p.h.l4 == L4_TCP) { sp = p.h.tcp.sport; dpp = p.h.tcp.dport; }
  if (p.h.l4 == L4_UDP) { sp = p.h.udp.sport; dpp = p.h.udp.dport; }
  const uint8_t *src = p.h.net == 4 ? p.h.v4.src : p.h.v6.src;
  const uint8_t *dst = p.h.net == 4 ? p.h.v4.dst : p.h.v6.dst;
  const auto &tab = p.h.net == 4 ? T.acl4 : T.acl6;
  Key k{proto, p.m.src_vni, p.m.dst_vni, 0, src, dst, sp, dpp};
  int64_t ri = classify(tab, k, p.h.net);
  // packet_has_valid_flow (acl-filter/src/lib.rs:71-94)
  const bool valid_flow = FL && p.flow >= 0 && FL->f[p.flow].status == DP_FLOW_ACTIVE &&
                          FL->f[p.flow].d.genid >= T.genid;
  int64_t rr = -1;
  const std::vector<Rule> *rtab = nullptr;
  if (ri < 0 && valid_flow && flow_alive(FL, FL->f[p.flow].related)) {
    // reverse_summary (lib.rs:205-217): the related flow's key between the
    // swapped VPCs; a Flow-scope Allow admits the reply (lib.rs:110-128)
    const FKey &rk = FL->f[FL->f[p.flow].related].key;
    const uint8_t rproto = rk.kind == DP_FLOW_TCP ? 6 : rk.kind == DP_FLOW_UDP ? 17 : rk.fam == 4 ? 1 : 58;
    const bool rports = rk.kind == DP_FLOW_TCP || rk.kind == DP_FLOW_UDP;
    rtab = rk.fam == 4 ? &T.acl4 : &T.acl6;
    Key rkey{rproto, p.m.dst_vni, p.m.src_vni, 0, rk.src, rk.dst, (uint16_t)(rports ? rk.sp : 0),
             (uint16_t)(rports ? rk.dp : 0)};
    rr = classify(*rtab, rkey, rk.fam);
    if (rr >= 0 && !((*rtab)[rr].r.action == DP_ACL_ALLOW && (*rtab)[rr].r.action2 == DP_ACL_SCOPE_FLOW))
      rr = -1;
  }
  uint32_t action;
  if (ri >= 0) {
    action = tab[ri].r.action;
    p.m.acl_rule = tab[ri].orig_index;
    p.m.acl = action == DP_ACL_DENY ? 2 : 1;
  } else if (rr >= 0) {
    action = DP_ACL_ALLOW;
    p.m.acl_rule = (*rtab)[rr].orig_index;
    p.m.acl = 6;
  } else {
    auto it = T.acl_default.find({p.m.src_vni, p.m.dst_vni});
    if (it != T.acl_default.end()) {
      action = it->second;
      p.m.acl = action == DP_ACL_DENY ? 4 : 3;
    } else {
      action = DP_ACL_ALLOW;
      p.m.acl = 5;
    }
  }
  if (action == DP_ACL_DENY) {
    flow_invalidate_pair(FL, p.flow);
    p.done(DP_DONE_ACL_DROPPED);
  }
}

// Embedded transport ports (EmbeddedTransport::source / destination,
// embedded.rs:545-601): TCP / UDP only, full or partial headers alike.
bool emb_port(const Emb &e, bool src, uint16_t &port) {
  if (e.tk != L4_TCP && e.tk != L4_UDP) return false;
  if (!e.full) port = be16(e.part.data() + (src ? 0 : 2));
  else if (e.tk == L4_TCP) port = src ? e.tcp.sport : e.tcp.dport;
  else port = src ? e.udp.sport : e.udp.dport;
  return true;
}
// set_source / set_destination of the embedded transport.  The reference
// also calls update_checksum on it, but discards the incremental result
// (icmp_error_msg.rs translate_inner_tcp_udp_*, embedded.rs:612-647, the
// default Checksum::increment_update_checksum returns, never stores): the
// embedded transport checksum stays as it was.
void emb_set_port(Emb &e, bool src, uint16_t port) {
  if (!e.full) put16(e.part.data() + (src ? 0 : 2), port);
  else if (e.tk == L4_TCP) (src ? e.tcp.sport : e.tcp.dport) = port;
  else (src ? e.udp.sport : e.udp.dport) = port;
}

// StaticNat (nat/src/static_nat/nf.rs:158-368), with the embedded packet of
// an ICMP error message translated back (nf.rs:111-155,
// nat/src/icmp_handler/icmp_error_msg.rs: nat_translate_icmp_inner_src/dst)
void stage_static_nat(const dpo_tables &T, Packet &p) {
  if (p.is_done()) return;
  uint32_t need = DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST;
  if (!(p.m.flags & need)) return;
  const bool icmp_err = icmp_is_error_msg(p.h) && p.h.emb.present;
  // an ICMP error message is NATed even when already marked NATed (nf.rs:350-362)
  if ((p.m.flags & (DP_META_NATTED_SRC | DP_META_NATTED_DST)) && !icmp_err) return;
  if (!p.m.src_vni || !p.m.dst_vni) { p.done(DP_DONE_UNROUTABLE); return; }
  auto dt = T.nat_dst.find(p.m.src_vni);
  bool has_src_tables = false;
  for (auto &kv : T.nat_src) if (kv.first.first == p.m.src_vni) { has_src_tables = true; break; }
  if (dt == T.nat_dst.end() && !has_src_tables) { p.done(DP_DONE_UNROUTABLE); return; }  // MissingTable
  if (p.h.net == 0) { p.done(DP_DONE_NOT_IP); return; }
  bool modified = false;
  bool has_sp = p.h.l4 == L4_TCP || p.h.l4 == L4_UDP;
  uint16_t *psp = p.h.l4 == L4_TCP ? &p.h.tcp.sport : &p.h.udp.sport;
  uint16_t *pdp = p.h.l4 == L4_TCP ? &p.h.tcp.dport : &p.h.udp.dport;
  Emb &e = p.h.emb;
  auto st = T.nat_src.find({p.m.src_vni, p.m.dst_vni});
  if ((p.m.flags & DP_META_REQ_STATIC_NAT_SRC) && !(p.m.flags & DP_META_NATTED_SRC)) {
    bool mod = false;
    if (st != T.nat_src.end() && p.h.net == 4) {
      uint32_t na; bool hp; uint16_t np;
      if (nat_find_mapping(st->second, p.h.v4.src, has_sp, has_sp ? *psp : 0, na, hp, np)) {
        // UnicastIpAddr::try_from: not multicast / broadcast
        bool unicast = !((na >> 28) == 0xe || na == 0xffffffffu);
        if (unicast) {
          if (na != be32(p.h.v4.src)) { put32(p.h.v4.src, na); mod = true; }
          if (has_sp && hp && np != *psp) { *psp = np; mod = true; }
        }
      }
    }
    // the embedded packet's destination: find_src_mapping (nf.rs:134-155)
    if (icmp_err && st != T.nat_src.end() && e.net == 4) {
      uint16_t port = 0;
      const bool hp_in = emb_port(e, false, port);
      uint32_t na; bool hp; uint16_t np;
      if (nat_find_mapping(st->second, e.v4.dst, hp_in, port, na, hp, np) &&
          !((na >> 28) == 0xe || na == 0xffffffffu)) {
        put32(e.v4.dst, na);
        if (hp_in && hp) emb_set_port(e, false, np);
        mod = true;  // Ok(true) whenever a mapping exists
      }
    }
    if (mod) p.m.flags |= DP_META_NATTED_SRC;
    modified |= mod;
  }
  if ((p.m.flags & DP_META_REQ_STATIC_NAT_DST) && !(p.m.flags & DP_META_NATTED_DST)) {
    bool mod = false;
    if (dt != T.nat_dst.end() && p.h.net == 4) {
      uint32_t na; bool hp; uint16_t np;
      if (nat_find_mapping(dt->second, p.h.v4.dst, has_sp, has_sp ? *pdp : 0, na, hp, np)) {
        if (na != be32(p.h.v4.dst)) { put32(p.h.v4.dst, na); mod = true; }
        if (has_sp && hp && np != *pdp) { *pdp = np; mod = true; }
      }
    }
    // the embedded packet's source: find_dst_mapping (nf.rs:111-132); a
    // non-unicast target is NotUnicast -> NatFailure (icmp_error_msg.rs)
    if (icmp_err && dt != T.nat_dst.end() && e.net == 4) {
      uint16_t port = 0;
      const bool hp_in = emb_port(e, true, port);
      uint32_t na; bool hp; uint16_t np;
      if (nat_find_mapping(dt->second, e.v4.src, hp_in, port, na, hp, np)) {
        if ((na >> 28) == 0xe || na == 0xffffffffu) { p.done(DP_DONE_NAT_FAILURE); return; }
        put32(e.v4.src, na);
        if (hp_in && hp) emb_set_port(e, true, np);
        mod = true;
      }
    }
    if (mod) p.m.flags |= DP_META_NATTED_DST;
    modified |= mod;
  }
  if (modified) p.m.flags |= DP_META_REFR_CHKSUM;
}


// ---------------------------------------------------------------------------
// Port forwarding (nat/src/portfw/)
// ---------------------------------------------------------------------------
int32_t flow_insert_one(dpo_flows *FL, const dp_flow_t &d, int64_t partner, int64_t &ref);

bool same_prefix(const dp_prefix_t &a, const dp_prefix_t &b) {
  return a.family == b.family && a.len == b.len && memcmp(a.addr, b.addr, a.family == 4 ? 4 : 16) == 0;
}
// PortFwEntry::matches (objects.rs:159-166): everything but the timeouts
bool pf_matches(const dp_portfw_rule_t &a, const dp_portfw_rule_t &b) {
  return a.src_vni == b.src_vni && a.proto == b.proto && same_prefix(a.ext_prefix, b.ext_prefix) &&
         same_prefix(a.int_prefix, b.int_prefix) && a.ext_lo == b.ext_lo && a.ext_hi == b.ext_hi &&
         a.int_lo == b.int_lo && a.int_hi == b.int_hi && a.dst_vni == b.dst_vni;
}
uint64_t pf_init_ns(const dp_portfw_rule_t &r) {  // DEFAULT_INITIAL_TOUT (objects.rs:50)
  return (uint64_t)(r.init_timeout_s ? r.init_timeout_s : 10) * 1000000000ull;
}
uint64_t pf_estab_ns(const dp_portfw_rule_t &r) {  // DEFAULT_ESTABLISHED_TOUT_TCP / _UDP (:51-52)
  return (uint64_t)(r.estab_timeout_s ? r.estab_timeout_s : (r.proto == 6 ? 1800 : 30)) * 1000000000ull;
}
// PortFwTable::update (objects.rs:284-300): entries absent from the new rule
// set are removed; the rules are then added last to first (add_entry,
// :256-274): one that matches an entry at its (key, prefix, port range)
// keeps that entry (new timeouts), one whose range overlaps another of the
// same key and prefix is refused (RangeSet::insert_range, rangeset.rs:73-79).
void pf_update(dpo_tables &T, const dpo_tables *prev, const dp_portfw_rule_t *rs, uint32_t n) {
  T.pf_next_id = prev ? prev->pf_next_id : 1;
  if (prev)
    for (const PfRule &e : prev->pf) {
      bool keep = false;
      for (uint32_t i = 0; i < n && !keep; i++) keep = pf_matches(e.r, rs[i]);
      if (keep) T.pf.push_back(e);
    }
  for (uint32_t k = n; k-- > 0;) {
    const dp_portfw_rule_t &r = rs[k];
    PfRule *exist = nullptr;
    bool overlap = false;
    for (PfRule &e : T.pf) {
      if (e.r.src_vni != r.src_vni || e.r.proto != r.proto || !same_prefix(e.r.ext_prefix, r.ext_prefix)) continue;
      if (e.r.ext_lo == r.ext_lo && e.r.ext_hi == r.ext_hi) exist = &e;
      if (e.r.ext_lo <= r.ext_hi && r.ext_lo <= e.r.ext_hi) overlap = true;
    }
    if (exist && pf_matches(exist->r, r)) {
      exist->r.init_timeout_s = r.init_timeout_s;
      exist->r.estab_timeout_s = r.estab_timeout_s;
      exist->init_ns = pf_init_ns(r);
      exist->estab_ns = pf_estab_ns(r);
      continue;
    }
    if (overlap) continue;  // "Failure adding port-forwarding rule"
    T.pf.push_back(PfRule{r, T.pf_next_id++, pf_init_ns(r), pf_estab_ns(r)});
  }
}
// PortFwEntry::new's checks (objects.rs:70-155, portrange.rs:33-42)
bool pf_valid(const dp_portfw_rule_t &r) {
  if (r.proto != 6 && r.proto != 17) return false;
  if (r.ext_prefix.family != r.int_prefix.family || r.ext_prefix.len != r.int_prefix.len) return false;
  if (r.src_vni == r.dst_vni || !r.src_vni || !r.dst_vni) return false;
  if (!r.ext_lo || !r.int_lo || r.ext_hi < r.ext_lo || r.int_hi < r.int_lo) return false;
  return r.ext_hi - r.ext_lo == r.int_hi - r.int_lo;
}
const PfRule *pf_by_id(const dpo_tables &T, uint32_t id) {  // Weak::upgrade of an entry
  for (const PfRule &e : T.pf) if (e.id == id) return &e;
  return nullptr;
}
// PortFwTable::lookup_matching_rule -> LpmMap::lookup_cumulative
// (objects.rs:304-313, lpmmap.rs:108-116): of the key's prefixes holding the
// address, longest first, the first whose port ranges hold the port
const PfRule *pf_lookup(const dpo_tables &T, uint32_t src_vni, uint8_t proto, const Ip &a, uint16_t port) {
  const PfRule *best = nullptr;
  for (const PfRule &e : T.pf) {
    if (e.r.src_vni != src_vni || e.r.proto != proto || e.r.ext_prefix.family != a.fam) continue;
    if (!prefix_covers(e.r.ext_prefix.addr, e.r.ext_prefix.len, a.b)) continue;
    if (port < e.r.ext_lo || port > e.r.ext_hi) continue;
    if (!best || e.r.ext_prefix.len > best->r.ext_prefix.len) best = &e;
  }
  return best;
}
bool ip_unicast(const Ip &a) {  // UnicastIpv4Addr / UnicastIpv6Addr::new
  if (a.fam == 4) return !((a.b[0] >> 4) == 0xe || (a.b[0] == 255 && a.b[1] == 255 && a.b[2] == 255 && a.b[3] == 255));
  return a.b[0] != 0xff;
}
// PortFwEntry::map_address_port (objects.rs:168-203): the port's index in
// ext_ports into int_ports; the address's offset from the external network
// onto the internal one (wrapping integer arithmetic); a unicast result
bool pf_map(const PfRule &e, const Ip &a, uint16_t port, Ip &na, uint16_t &np) {
  if (port < e.r.ext_lo || port > e.r.ext_hi) return false;
  np = (uint16_t)(e.r.int_lo + (port - e.r.ext_lo));
  na = Ip{};
  na.fam = a.fam;
  const int nb = a.fam == 4 ? 4 : 16;
  int carry = 0, borrow = 0;
  uint8_t off[16];
  for (int i = nb - 1; i >= 0; i--) {  // offset = address - ext network
    int d = (int)a.b[i] - e.r.ext_prefix.addr[i] - borrow;
    borrow = d < 0;
    off[i] = (uint8_t)(d + (borrow ? 256 : 0));
  }
  for (int i = nb - 1; i >= 0; i--) {  // int network + offset
    int v = (int)e.r.int_prefix.addr[i] + off[i] + carry;
    carry = v > 255;
    na.b[i] = (uint8_t)v;
  }
  return ip_unicast(na);
}
Ip pkt_src(const Packet &p) { return p.h.net == 4 ? ip4(p.h.v4.src) : ip6(p.h.v6.src); }
Ip pkt_dst(const Packet &p) { return p.h.net == 4 ? ip4(p.h.v4.dst) : ip6(p.h.v6.dst); }
uint8_t pkt_proto(const Packet &p) { return p.h.net == 4 ? p.h.v4.proto : p.h.v6.nh; }
bool pkt_ports(const Packet &p, uint16_t &sp, uint16_t &dpp) {  // transport src / dst port
  if (p.h.l4 == L4_TCP) { sp = p.h.tcp.sport; dpp = p.h.tcp.dport; return true; }
  if (p.h.l4 == L4_UDP) { sp = p.h.udp.sport; dpp = p.h.udp.dport; return true; }
  return false;
}
void set_ip(Packet &p, bool src, const Ip &a) {
  uint8_t *q = p.h.net == 4 ? (src ? p.h.v4.src : p.h.v4.dst) : (src ? p.h.v6.src : p.h.v6.dst);
  memcpy(q, a.b, p.h.net == 4 ? 4 : 16);
}
// nat_packet (portfw/packet.rs:42-154): DstNat rewrites the destination
// address and port, SrcNat the source; an ICMP packet only its address.
// false: unsupported traffic (-> InternalFailure)
bool pf_nat_packet(Packet &p, uint8_t action, const Ip &a, uint16_t port) {
  const bool src = action == DP_PF_SRC_NAT;
  if (p.h.net == 0 || a.fam != p.h.net) return false;
  const uint8_t proto = pkt_proto(p);
  bool mod = false;
  if ((proto == 6 || proto == 17) && (p.h.l4 == L4_TCP || p.h.l4 == L4_UDP)) {
    Ip cur = src ? pkt_src(p) : pkt_dst(p);
    if (!(cur == a)) { set_ip(p, src, a); mod = true; }
    uint16_t *pp = p.h.l4 == L4_TCP ? (src ? &p.h.tcp.sport : &p.h.tcp.dport)
                                    : (src ? &p.h.udp.sport : &p.h.udp.dport);
    if (*pp != port) { *pp = port; mod = true; }
  } else if ((p.h.net == 4 ? proto == 1 && p.h.l4 == L4_ICMP4 : proto == 58 && p.h.l4 == L4_ICMP6)) {
    Ip cur = src ? pkt_src(p) : pkt_dst(p);
    if (!(cur == a)) { set_ip(p, src, a); mod = true; }
  } else {
    return false;
  }
  if (mod) p.m.flags |= DP_META_REFR_CHKSUM | (src ? DP_META_NATTED_SRC : DP_META_NATTED_DST);
  return true;
}
// get_rule_from_pkt (portfw/nf.rs:206-324): is the stale state of this flow
// still what the current rules would do?  The entry, or null.
const PfRule *pf_rule_from_pkt(const dpo_tables &T, const Packet &p, const OFlow &f) {
  uint16_t sp, dpp;
  if (!p.m.src_vni || p.h.net == 0 || !pkt_ports(p, sp, dpp)) return nullptr;
  const uint8_t proto = pkt_proto(p);
  if (f.pf == DP_PF_DST_NAT) {  // forward path (:206-244)
    const PfRule *e = pf_lookup(T, p.m.src_vni, proto, pkt_dst(p), dpp);
    Ip na; uint16_t np;
    if (!e || !pf_map(*e, pkt_dst(p), dpp, na, np)) return nullptr;
    if (!(na == f.pf_ip) || np != f.pf_port || e->r.dst_vni != f.d.dst_vni) return nullptr;
    return e;
  }
  // reverse path (:246-288)
  const PfRule *e = pf_lookup(T, f.d.dst_vni, proto, f.pf_ip, f.pf_port);
  Ip ta; uint16_t tp;
  if (!e || !pf_map(*e, f.pf_ip, f.pf_port, ta, tp)) return nullptr;
  if (!(ta == pkt_src(p)) || tp != sp || e->r.dst_vni != p.m.src_vni) return nullptr;
  return e;
}
// next_flow_status (portfw/protocol.rs:17-69)
uint8_t pf_next_status(const Packet &p, uint8_t action, uint8_t st) {
  if (p.h.l4 == L4_TCP) {
    const uint8_t fl = p.h.tcp.flags;
    const bool fin = fl & 0x01, syn = fl & 0x02, rst = fl & 0x04, ack = fl & 0x10;
    if (action == DP_PF_DST_NAT) {
      if (st == DP_NFS_TWO_WAY && !syn && ack) return DP_NFS_ESTABLISHED;
      if (st == DP_NFS_ESTABLISHED && fin) return DP_NFS_C_CLOSING;
      if (st == DP_NFS_S_CLOSING && !fin && ack) return DP_NFS_S_HALF_CLOSE;
      if (st == DP_NFS_S_CLOSING && fin && ack) return DP_NFS_LAST_ACK;
      if (st == DP_NFS_S_HALF_CLOSE && fin) return DP_NFS_LAST_ACK;
      if (st == DP_NFS_LAST_ACK && ack) return DP_NFS_CLOSED;
    } else {
      if (st == DP_NFS_ONE_WAY && syn && ack) return DP_NFS_TWO_WAY;
      if (st == DP_NFS_ESTABLISHED && fin) return DP_NFS_S_CLOSING;
      if (st == DP_NFS_C_CLOSING && !fin && ack) return DP_NFS_C_HALF_CLOSE;
      if (st == DP_NFS_C_CLOSING && fin && ack) return DP_NFS_LAST_ACK;
      if (st == DP_NFS_C_HALF_CLOSE && fin) return DP_NFS_LAST_ACK;
      if (st == DP_NFS_LAST_ACK && ack) return DP_NFS_CLOSED;
    }
    return rst ? (uint8_t)DP_NFS_RESET : st;
  }
  if (action == DP_PF_DST_NAT) return st == DP_NFS_TWO_WAY ? (uint8_t)DP_NFS_ESTABLISHED : st;
  return st == DP_NFS_ONE_WAY ? (uint8_t)DP_NFS_TWO_WAY : st;
}
// FlowInfo::reset_expiry_unchecked (flow_info.rs:399-407)
void reset_expiry(OFlow &f, uint64_t now, uint64_t dur) {
  const uint64_t nw = now + dur;
  if (nw >= f.d.expires_at) f.d.expires_at = nw;
}
// refresh_port_fw_entry (portfw/flow_state.rs:216-264)
void pf_refresh(const dpo_tables &T, dpo_flows *FL, Packet &p, const PfRule &e, int64_t fi) {
  OFlow &f = FL->f[fi];
  uint8_t &st = FL->nfs[f.pf_status];
  const uint8_t cur = st, nw = pf_next_status(p, f.pf, cur);
  st = nw;
  uint64_t ext;
  if (nw == DP_NFS_ESTABLISHED) ext = e.estab_ns;
  else if (nw == DP_NFS_CLOSED || nw == DP_NFS_RESET) { flow_invalidate_pair(FL, fi); return; }
  else ext = e.init_ns;
  reset_expiry(f, FL->now, ext);
  if (nw == DP_NFS_ESTABLISHED && nw != cur && flow_alive(FL, f.related))
    reset_expiry(FL->f[f.related], FL->now, ext);
  f.d.genid = T.genid;
}
// FlowInfo::related_pair + insert_from_arc of both (portfw/nf.rs:96-172)
void pf_create(const dpo_tables &T, dpo_flows *FL, Packet &p, const PfRule &e, const Ip &dst,
               uint16_t dport, const Ip &na, uint16_t np) {
  FKey cur;
  uint16_t sp, dpp;
  if (!packet_flow_key(p, cur) || !pkt_ports(p, sp, dpp)) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
  const FKey fwk = p.has_ikey ? p.ikey : cur;  // build_portfw_flow_keys (flow_state.rs:102-131)
  FKey rk;                                     // (current key DNATed).reverse(dst_vpcd)
  rk.vni = e.r.dst_vni;
  rk.fam = cur.fam;
  rk.kind = cur.kind;
  memcpy(rk.src, na.b, 16);
  if (na.fam == 4) memset(rk.src + 4, 0, 12);
  memcpy(rk.dst, cur.src, 16);
  rk.sp = np;
  rk.dp = cur.sp;
  if (fwk == rk) { p.done(DP_DONE_INTERNAL_FAILURE); return; }  // related_pair: identical keys
  dp_flow_t fd{}, rd{};
  auto to_key = [](const FKey &k, dp_flow_key_t &x) {
    x.src_vni = k.vni; x.family = k.fam; x.kind = k.kind; x.sport = k.sp; x.dport = k.dp;
    memcpy(x.src, k.src, 16); memcpy(x.dst, k.dst, 16);
  };
  to_key(fwk, fd.key);
  to_key(rk, rd.key);
  // compute_flow_flags_forward / _reverse (net/src/packet/meta.rs:264-287)
  fd.flags = DP_FLOW_INITIATOR;
  if (p.m.flags & DP_META_REQ_STATIC_NAT_SRC) { fd.flags |= DP_FLOW_REQ_STATIC_NAT_SRC; rd.flags |= DP_FLOW_REQ_STATIC_NAT_DST; }
  if (p.m.flags & DP_META_REQ_STATIC_NAT_DST) { fd.flags |= DP_FLOW_REQ_STATIC_NAT_DST; rd.flags |= DP_FLOW_REQ_STATIC_NAT_SRC; }
  fd.dst_vni = e.r.dst_vni;   // setup_forward_flow (flow_state.rs:133-157)
  rd.dst_vni = e.r.src_vni;   // setup_reverse_flow (:159-177)
  fd.genid = rd.genid = T.genid;  // set_genid_pair
  fd.expires_at = rd.expires_at = FL->now + e.init_ns;
  // the DNAT of this packet, before any insert (nf.rs:144-150)
  if (!pf_nat_packet(p, DP_PF_DST_NAT, na, np)) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
  const int64_t cell = (int64_t)FL->nfs.size();
  FL->nfs.push_back(DP_NFS_ONE_WAY);
  int64_t rf, rr;
  // the forward insert: its related flow is not in the table yet
  if (flow_insert_one(FL, fd, -1, rf) < 0) { p.done(DP_DONE_FLOW_CAPACITY_EXCEEDED); return; }
  OFlow *F = &FL->f[rf];
  F->pf = DP_PF_DST_NAT; F->pf_status = cell; F->pf_ip = na; F->pf_port = np; F->pf_rule = e.id;
  if (flow_insert_one(FL, rd, rf, rr) < 0) {  // admitted at capacity: its related flow is Active
    flow_invalidate(FL, rf);
    p.done(DP_DONE_FLOW_CAPACITY_EXCEEDED);
    return;
  }
  OFlow &R = FL->f[rr];
  R.pf = DP_PF_SRC_NAT; R.pf_status = cell; R.pf_ip = dst; R.pf_port = dport; R.pf_rule = e.id;
  FL->f[rf].related = rr;
  R.related = rf;
}
// PortForwarder (portfw/nf.rs:326-397)
void stage_portfw(const dpo_tables &T, dpo_flows *FL, Packet &p) {
  if (p.is_done() || !(p.m.flags & DP_META_REQ_PORT_FORWARDING) || icmp_is_error_msg(p.h)) return;
  if (!FL) { p.done(DP_DONE_INTERNAL_FAILURE); return; }  // its Arc<FlowTable> is not optional
  // get_packet_port_fw_state (flow_state.rs:181-204): an Active flow with state
  if (p.flow >= 0 && FL->f[p.flow].status == DP_FLOW_ACTIVE && FL->f[p.flow].pf != DP_PF_NONE) {
    OFlow &f = FL->f[p.flow];
    const PfRule *e = pf_by_id(T, f.pf_rule);
    if (!e) {  // a stale rule: would the current rules still do this?
      e = pf_rule_from_pkt(T, p, f);
      if (!e) {
        p.done(DP_DONE_NAT_NOT_PORT_FORWARDED);
        flow_invalidate_pair(FL, p.flow);
        return;
      }
      f.pf_rule = e->id;  // reassign_port_fw_rule, both flows (nf.rs:290-320)
      if (flow_alive(FL, f.related)) FL->f[f.related].pf_rule = e->id;
    }
    if (!pf_nat_packet(p, f.pf, f.pf_ip, f.pf_port)) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
    pf_refresh(T, FL, p, *e, p.flow);
    return;
  }
  // try_port_forwarding (nf.rs:174-204); can_be_port_forwarded (:54-94)
  if (!p.m.src_vni) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
  uint16_t sp, dpp;
  if (!p.h.has_eth || p.h.net == 0 || !pkt_ports(p, sp, dpp)) { p.done(DP_DONE_NAT_NOT_PORT_FORWARDED); return; }
  if (p.h.l4 == L4_TCP) {  // Tcp::is_first_segment (net/src/tcp/mod.rs:310-312)
    const uint8_t fl = p.h.tcp.flags;
    if (!((fl & 0x02) && !(fl & 0x3d))) { p.done(DP_DONE_NAT_NOT_PORT_FORWARDED); return; }
  }
  const Ip dst = pkt_dst(p);
  if (!ip_unicast(dst)) { p.done(DP_DONE_NAT_NOT_PORT_FORWARDED); return; }
  const PfRule *e = pf_lookup(T, p.m.src_vni, pkt_proto(p), dst, dpp);
  if (!e) { p.done(DP_DONE_NAT_NOT_PORT_FORWARDED); return; }
  Ip na;
  uint16_t np;
  if (!pf_map(*e, dst, dpp, na, np)) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
  pf_create(T, FL, p, *e, dst, dpp, na, np);
}

// ---------------------------------------------------------------------------
// Masquerade (nat/src/masquerade/nf.rs)
// ---------------------------------------------------------------------------
const uint64_t kMasqOneWayNs = 5000000000ull;   // MASQUERADE_ONEWAY_TIMEOUT (nf.rs:86)
const uint64_t kMasqTwoWayNs = 3000000000ull;   // MASQUERADE_TWOWAY_TIMEOUT (:87)
const uint64_t kMasqClosingNs = 2000000000ull;  // MASQUERADE_CLOSING_TIMEOUT (:88)

// masquerade (packet.rs:35-195): the snat / dnat of a state -- the address,
// and a TCP / UDP port (always, NatPort::Port) or an ICMP query identifier
// (when it changes).  false: the error (UnusableAddress, UnsupportedTraffic,
// a header of the other family).
bool masq_xlate(Packet &p, uint8_t action, const Ip &a, uint16_t port, bool ident) {
  const bool src = action == DP_PF_SRC_NAT;
  if (src && !ip_unicast(a)) return false;  // UnicastIpAddr::try_from
  if (!p.h.has_eth || p.h.net == 0) return false;
  bool mod = false;
  auto set_addr = [&]() -> bool {
    if (a.fam != p.h.net) return false;  // NetError
    const Ip cur = src ? pkt_src(p) : pkt_dst(p);
    if (!(cur == a)) { set_ip(p, src, a); mod = true; }
    return true;
  };
  if (p.h.l4 == L4_TCP || p.h.l4 == L4_UDP) {
    if (!set_addr()) return false;
    if (!ident) {
      uint16_t *pp = p.h.l4 == L4_TCP ? (src ? &p.h.tcp.sport : &p.h.tcp.dport)
                                      : (src ? &p.h.udp.sport : &p.h.udp.dport);
      *pp = port;
      mod = true;
    }
  } else if (p.h.l4 == L4_ICMP4 || p.h.l4 == L4_ICMP6) {
    if (!set_addr()) return false;
    uint16_t cur;
    if (ident && icmp_full_identifier(p.h.icmp, p.h.l4 == L4_ICMP6, cur) && cur != port) {
      put16(p.h.icmp.raw + 4, port);
      mod = true;
    }
  } else {
    return false;
  }
  if (mod) p.m.flags |= DP_META_REFR_CHKSUM | (src ? DP_META_NATTED_SRC : DP_META_NATTED_DST);
  return true;
}

// next_flow_status (masquerade/protocol.rs:93-116) on the IP header's next
// header: TCP by its flags, UDP (a DstNat reply from port 53 / 853 / 8853
// closes), ICMP
uint8_t masq_next_status(const Packet &p, uint8_t action, uint8_t st) {
  const uint8_t proto = pkt_proto(p);
  const bool snat = action == DP_PF_SRC_NAT;
  if (proto == 17) {
    uint8_t n = st;
    if (snat) { if (st == DP_NFS_TWO_WAY) n = DP_NFS_ESTABLISHED; }
    else if (st == DP_NFS_ONE_WAY) n = DP_NFS_TWO_WAY;
    if (!snat && p.h.has_eth && p.h.l4 == L4_UDP) {
      const uint16_t sp = p.h.udp.sport;
      if (sp == 53 || sp == 853 || sp == 8853) n = DP_NFS_CLOSED;
    }
    return n;
  }
  if (proto == 1 || proto == 58) return (!snat && st == DP_NFS_ONE_WAY) ? (uint8_t)DP_NFS_TWO_WAY : st;
  if (proto == 6 && p.h.l4 == L4_TCP)
    // the same machine as port forwarding's, the initiator's side being SrcNat here
    return pf_next_status(p, snat ? (uint8_t)DP_PF_DST_NAT : (uint8_t)DP_PF_SRC_NAT, st);
  return st;
}

// refresh_masquerade_state (nf.rs:151-194)
void masq_refresh(dpo_flows *FL, Packet &p, int64_t fi) {
  OFlow &f = FL->f[fi];
  uint8_t &st = FL->nfs[f.m_status];
  const uint8_t cur = st, nw = masq_next_status(p, f.masq, cur);
  st = nw;
  uint64_t ext = 0;
  switch (nw) {
    case DP_NFS_TWO_WAY: ext = kMasqTwoWayNs; break;
    case DP_NFS_ESTABLISHED: ext = f.m_idle_ns; break;
    case DP_NFS_CLOSED: case DP_NFS_RESET: flow_invalidate_pair(FL, fi); return;
    case DP_NFS_ONE_WAY: return;
    default: ext = kMasqClosingNs; break;
  }
  reset_expiry(f, FL->now, ext);
  if (cur != nw && nw == DP_NFS_ESTABLISHED && flow_alive(FL, f.related))
    reset_expiry(FL->f[f.related], FL->now, ext);
}

uint8_t key_proto(const FKey &k) {  // FlowKey::proto (flow_key.rs:536-548)
  if (k.kind == DP_FLOW_TCP) return 6;
  if (k.kind == DP_FLOW_UDP) return 17;
  return k.fam == 4 ? 1 : 58;
}
Ip key_src(const FKey &k) { Ip a; a.fam = k.fam; memcpy(a.b, k.src, 16); if (k.fam == 4) memset(a.b + 4, 0, 12); return a; }

// Masquerade::masquerade_packet (nf.rs:384-475); returns the DoneReason of the
// error (MasqueradeError -> DoneReason, nf.rs:547-568) or -1
int masq_packet(const dpo_tables &T, dpo_flows *FL, Packet &p) {
  // get_masquerade_state (nf.rs:198-213): an Active flow with masquerade state
  if (p.flow >= 0 && FL->f[p.flow].status == DP_FLOW_ACTIVE && FL->f[p.flow].masq != DP_PF_NONE) {
    OFlow &f = FL->f[p.flow];
    const uint8_t act = f.masq;
    const Ip ip = f.m_ip;
    const uint16_t port = f.m_port;
    const bool ident = f.m_ident;
    masq_refresh(FL, p, p.flow);
    return masq_xlate(p, act, ip, port, ident) ? -1 : DP_DONE_NAT_FAILURE;
  }
  const std::shared_ptr<MAlloc> A = FL->alloc;
  if (!A) return DP_DONE_NAT_FAILURE;  // NoAllocator
  if (p.h.l4 == L4_TCP) {  // "TCP without SYN": Tcp::is_first_segment
    const uint8_t fl = p.h.tcp.flags;
    if (!((fl & 0x02) && !(fl & 0x3d))) return DP_DONE_FILTERED;
  }
  FKey cur;
  if (!packet_flow_key(p, cur)) return DP_DONE_MALFORMED;  // FlowKeyError
  const FKey init = p.has_ikey ? p.ikey : cur;
  const uint8_t proto = key_proto(init);
  // NatAllocator::allocate (apalloc/mod.rs:317-375)
  const Ip sip = key_src(init);
  const MPoolSet *S = A->lookup(init.fam, proto, p.m.src_vni, p.m.dst_vni, addr_bits(init.fam, sip.b));
  if (!S) return DP_DONE_FILTERED;  // Denied
  std::shared_ptr<MPort> alloc;
  const MErr e = m_set_allocate(*S, proto == 1 || proto == 58, alloc);
  if (e != M_OK) return m_done(e);
  const Ip aip = alloc->ip();
  if (!ip_unicast(aip)) return DP_DONE_FILTERED;  // Bug("allocated unusable ip"); the allocation drops here
  // create_flow_pair (nf.rs:265-325): the reverse key from the current key
  // (new_reverse_session, :327-373), the original source (get_reverse_mapping)
  FKey rk;
  rk.vni = p.m.dst_vni;
  rk.fam = cur.fam;
  rk.kind = cur.kind;
  memcpy(rk.src, cur.dst, 16);
  memcpy(rk.dst, aip.b, 16);
  if (aip.fam == 4) memset(rk.dst + 4, 0, 12);
  if (cur.kind == DP_FLOW_TCP || cur.kind == DP_FLOW_UDP) {
    if (alloc->port == 0) return DP_DONE_MALFORMED;  // InvalidPort
    rk.sp = cur.dp;
    rk.dp = alloc->port;
  } else if (cur.kind == DP_FLOW_ICMP_QUERY) {
    rk.sp = alloc->port;
    rk.dp = 0;
  } else {
    return DP_DONE_NAT_FAILURE;  // UnexpectedKeyVariant
  }
  uint16_t rport;
  bool rident;
  if (init.kind == DP_FLOW_TCP || init.kind == DP_FLOW_UDP) { rport = init.sp; rident = false; }
  else if (init.kind == DP_FLOW_ICMP_QUERY) { rport = init.sp; rident = true; }
  else return DP_DONE_NAT_FAILURE;  // IcmpUnsupportedCategory
  if (init == rk) return DP_DONE_INTERNAL_FAILURE;  // related_pair: FlowInfoError
  dp_flow_t fd{}, rd{};
  auto to_key = [](const FKey &k, dp_flow_key_t &x) {
    x.src_vni = k.vni; x.family = k.fam; x.kind = k.kind; x.sport = k.sp; x.dport = k.dp;
    memcpy(x.src, k.src, 16); memcpy(x.dst, k.dst, 16);
  };
  to_key(init, fd.key);
  to_key(rk, rd.key);
  fd.flags = DP_FLOW_INITIATOR;
  if (p.m.flags & DP_META_REQ_STATIC_NAT_SRC) { fd.flags |= DP_FLOW_REQ_STATIC_NAT_SRC; rd.flags |= DP_FLOW_REQ_STATIC_NAT_DST; }
  if (p.m.flags & DP_META_REQ_STATIC_NAT_DST) { fd.flags |= DP_FLOW_REQ_STATIC_NAT_DST; rd.flags |= DP_FLOW_REQ_STATIC_NAT_SRC; }
  fd.dst_vni = p.m.dst_vni;   // setup_flow_masquerade_state: the forward flow goes to dst_vpcd,
  rd.dst_vni = p.m.src_vni;   // the reverse one to src_vpcd
  fd.genid = rd.genid = A->genid;  // set_genid_pair(allocator.genid())
  fd.expires_at = rd.expires_at = FL->now + kMasqOneWayNs;
  const int64_t cell = (int64_t)FL->nfs.size();
  FL->nfs.push_back(DP_NFS_ONE_WAY);
  int64_t rf, rr;
  if (flow_insert_one(FL, fd, -1, rf) < 0) return DP_DONE_FLOW_CAPACITY_EXCEEDED;  // the allocation drops here
  OFlow *F = &FL->f[rf];
  F->masq = DP_PF_SRC_NAT; F->m_status = cell; F->m_ip = aip; F->m_port = alloc->port;
  F->m_ident = alloc->ident; F->m_idle_ns = S->idle_ns; F->m_alloc = alloc;
  if (flow_insert_one(FL, rd, rf, rr) < 0) {  // admitted at capacity: its related flow is Active
    flow_invalidate(FL, rf);
    return DP_DONE_FLOW_CAPACITY_EXCEEDED;
  }
  OFlow &R = FL->f[rr];
  R.masq = DP_PF_DST_NAT; R.m_status = cell; R.m_ip = sip; R.m_port = rport; R.m_ident = rident;
  R.m_idle_ns = S->idle_ns;
  FL->f[rf].related = rr;
  R.related = rf;
  // the packet with the forward state; a failure invalidates the new pair
  if (!masq_xlate(p, DP_PF_SRC_NAT, aip, alloc->port, alloc->ident)) {
    flow_invalidate_pair(FL, rf);
    return DP_DONE_NAT_FAILURE;
  }
  return -1;  // recheck_flow: the allocator cannot change within a burst
}

// Masquerade::process (nf.rs:511-586)
void stage_masquerade(const dpo_tables &T, dpo_flows *FL, Packet &p) {
  if (p.is_done() || !(p.m.flags & DP_META_REQ_MASQUERADE) || icmp_is_error_msg(p.h)) return;
  if (!FL) { p.done(DP_DONE_INTERNAL_FAILURE); return; }  // its Arc<FlowTable> is not optional
  if (!p.m.src_vni || !p.m.dst_vni) { p.done(DP_DONE_UNROUTABLE); return; }
  if (p.h.net == 0) { p.done(DP_DONE_NOT_IP); return; }
  const int r = masq_packet(T, FL, p);
  if (r >= 0) p.done(r);
  else p.m.flags |= DP_META_REFR_CHKSUM;
}

// check_masquerading_flow (masquerade/flows.rs:94-174) for the flows of the
// table, then the allocator installed (update_nat_allocator,
// allocator_writer.rs:120-154).  The reference visits the flows in its
// DashMap's order; the restatement (and the GPU) re-reserve the carried
// allocations in ascending (address, port) order.
void masq_sync(const dpo_tables &T, dpo_flows *FL) {
  if (FL->synced == T.serial) return;
  FL->synced = T.serial;
  const std::shared_ptr<MAlloc> cur = FL->alloc;
  const bool same = cur && cur->randomize == T.masq_random && cur->seed == T.masq_seed &&
                    (cur->tag || T.masq_tag ? cur->tag == T.masq_tag && T.masq_tag != 0
                                            : cur->config == T.masq_cfg);
  if (same) {  // upgrade_all_masquerading_flows (flows.rs:30-44)
    cur->genid = T.genid;
    for (auto &kv : FL->map) {
      OFlow &f = FL->f[kv.second];
      if (f.status == DP_FLOW_ACTIVE && f.masq != DP_PF_NONE) f.d.genid = T.genid;
    }
    return;
  }
  if (T.masq.empty()) {  // invalidate_masquerade_flows (flows.rs:19-27)
    if (cur) {
      FL->alloc.reset();
      for (auto &kv : FL->map)
        if (FL->f[kv.second].masq != DP_PF_NONE) flow_invalidate_pair(FL, (int64_t)kv.second);
    }
    return;
  }
  auto A = m_build(T.masq, T.masq_cfg, T.masq_tag, T.genid, T.masq_random, T.masq_seed);
  std::vector<int64_t> fwd;
  for (auto &kv : FL->map) {
    const OFlow &f = FL->f[kv.second];
    if (f.status == DP_FLOW_ACTIVE && f.masq != DP_PF_NONE && f.d.genid != A->genid && f.m_alloc)
      fwd.push_back((int64_t)kv.second);
  }
  std::sort(fwd.begin(), fwd.end(), [&](int64_t a, int64_t b) {
    const OFlow &x = FL->f[a], &y = FL->f[b];
    const int c = memcmp(x.m_ip.b, y.m_ip.b, 16);
    if (c) return c < 0;
    return x.m_port < y.m_port;
  });
  for (int64_t fi : fwd) {
    OFlow &f = FL->f[fi];
    if (f.status != DP_FLOW_ACTIVE) continue;  // invalidated with an earlier flow of its pair
    const Ip &ip = f.m_ip;
    const Ip src = key_src(f.key);
    // find_masquerade_peering + the expose checks
    bool peering = false, ip_ok = false, compatible = false;
    for (auto &e : T.masq) {
      if (e.src_vni != f.key.vni || e.dst_vni != f.d.dst_vni) continue;
      peering = true;
      bool pub = false;
      for (auto &q : e.pub) pub |= q.family == ip.fam && prefix_covers(q.addr, q.len, ip.b);
      if (!pub) continue;
      ip_ok = true;
      bool pri = false;
      for (auto &q : e.priv) pri |= q.family == src.fam && prefix_covers(q.addr, q.len, src.b);
      if (pri) { compatible = true; break; }
    }
    if (!peering || !ip_ok || !compatible) { flow_invalidate_pair(FL, fi); continue; }
    // re_reserve_ip_and_port -> NatAllocator::reserve_port (apalloc/mod.rs:425-449)
    const MPoolSet *S = A->lookup(f.key.fam, key_proto(f.key), f.key.vni, f.d.dst_vni, addr_bits(src.fam, src.b));
    std::shared_ptr<MPort> np;
    if (!S || m_set_reserve(*S, ip, f.m_port, f.m_ident, np) != M_OK) { flow_invalidate_pair(FL, fi); continue; }
    f.m_alloc = np;  // the allocation from the replaced allocator drops
    f.d.genid = A->genid;  // set_genid_pair
    if (flow_alive(FL, f.related)) FL->f[f.related].d.genid = A->genid;
  }
  FL->alloc = A;
}

// IcmpErrorHandler (nat/src/icmp_handler/nf.rs:61-194) with an empty flow
// table: an overlay ICMP error message must carry an embedded IP header and
// transport (IcmpErrorPacket::new, net/src/packet/icmp_err.rs:37-53), valid
// ICMP and embedded IPv4 checksums (validate_checksums, :71-87) and a flow
// key (embedded ports, or an ICMP query identifier: flow_key.rs:635-660);
// then no flow is found and the packet goes on (nf.rs:113-120).
void stage_icmp_error(const dpo_tables &T, dpo_flows *FL, Packet &p) {
  if (p.is_done() || !p.overlay() || !icmp_is_error_msg(p.h)) return;
  const Emb &e = p.h.emb;
  if (!e.present || e.tk == L4_NONE) { p.done(DP_DONE_ICMP_ERROR_INCOMPLETE); return; }
  if (!p.m.src_vni) { p.done(DP_DONE_UNROUTABLE); return; }
  std::vector<uint8_t> v = icmp_checksum_payload(e, p.buf + p.pay_start, p.pay_end - p.pay_start);
  if (icmp_checksum(p.h, v.data(), v.size()) != be16(p.h.icmp.raw + 2)) {
    p.done(DP_DONE_INVALID_CHECKSUM);
    return;
  }
  if (e.net == 4 && ipv4_checksum(e.v4) != e.v4.csum) { p.done(DP_DONE_INVALID_CHECKSUM); return; }
  if (e.tk == L4_ICMP4 || e.tk == L4_ICMP6) {
    const bool v6 = e.tk == L4_ICMP6;
    bool has_id;
    uint16_t id;
    if (e.full) has_id = icmp_full_identifier(e.icmp, v6, id);
    else {
      // TruncatedIcmp4Header / TruncatedIcmp6Header::identifier: query type, >= 6 bytes
      const uint8_t t = e.part[0];
      const bool q = v6 ? (t == 128 || t == 129) : (t == 0 || t == 8 || t == 13 || t == 14);
      has_id = q && e.part.size() >= 6;
    }
    if (!has_id) { p.done(DP_DONE_ICMP_ERROR_INCOMPLETE); return; }  // EmbeddedMissingIcmpId
  }
  if (!FL) return;
  // the embedded packet's flow key, reversed, from the error's source VPC
  // (embedded_flowkey flow_key.rs:635-660, FlowKey::reverse :569-576)
  FKey k;
  k.vni = p.m.src_vni;
  if (e.net == 4) key_addrs(k, 4, e.v4.dst, e.v4.src);
  else key_addrs(k, 6, e.v6.dst, e.v6.src);
  if (e.tk == L4_TCP || e.tk == L4_UDP) {
    k.kind = e.tk == L4_TCP ? DP_FLOW_TCP : DP_FLOW_UDP;
    emb_port(e, false, k.sp);
    emb_port(e, true, k.dp);
  } else {
    k.kind = DP_FLOW_ICMP_QUERY;
    k.sp = e.full ? be16(e.icmp.raw + 4) : be16(e.part.data() + 4);
  }
  const int64_t r = flow_find(FL, k);
  if (r < 0) return;  // no flow: let the packet through (nf.rs:114-121)
  const OFlow &f = FL->f[r];
  if (f.status != DP_FLOW_ACTIVE) { p.done(DP_DONE_FILTERED); return; }  // nf.rs:126-130
  p.m.dst_vni = f.d.dst_vni;  // nf.rs:139-140
  if (f.masq != DP_PF_NONE) {
    // handle_icmp_error_masquerading (masquerade/icmp_handling.rs:16-48):
    // the embedded packet by reverse_translation_data (state.rs:89-98: SrcNat
    // its destination, DstNat its source, with the port or ICMP identifier),
    // then the error itself by the state; any failure is InternalFailure
    Emb &em = p.h.emb;
    const Ip &a = f.m_ip;
    const bool src = f.masq == DP_PF_DST_NAT;
    if (em.net != a.fam || (src && !ip_unicast(a))) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
    uint8_t *q = em.net == 4 ? (src ? em.v4.src : em.v4.dst) : (src ? em.v6.src : em.v6.dst);
    memcpy(q, a.b, a.fam == 4 ? 4 : 16);
    uint16_t old;
    if (emb_port(em, src, old)) {
      if (f.m_port == 0) { p.done(DP_DONE_INTERNAL_FAILURE); return; }  // InvalidPort
      if (old != f.m_port) emb_set_port(em, src, f.m_port);
    } else if (src && (em.tk == L4_ICMP4 || em.tk == L4_ICMP6)) {
      // translate_inner_icmp (icmp_error_msg.rs:149-173): the identifier, if
      // the embedded message has one (its checksum is left as it was)
      const bool v6 = em.tk == L4_ICMP6;
      uint16_t id;
      bool has;
      if (em.full) has = icmp_full_identifier(em.icmp, v6, id);
      else {
        const uint8_t t = em.part[0];
        has = (v6 ? (t == 128 || t == 129) : (t == 0 || t == 8 || t == 13 || t == 14)) && em.part.size() >= 6;
        if (has) id = be16(em.part.data() + 4);
      }
      if (has && id != f.m_port) {
        if (em.full) put16(em.icmp.raw + 4, f.m_port);
        else put16(em.part.data() + 4, f.m_port);
      }
    }
    if (!masq_xlate(p, f.masq, a, f.m_port, f.m_ident)) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
    const uint8_t t = p.h.icmp.raw[0], c = p.h.icmp.raw[1];
    const bool unrec = p.h.l4 == L4_ICMP4 ? (t == 3 && c != 4) : t == 1;
    if (unrec && FL->nfs[f.m_status] == DP_NFS_ONE_WAY) flow_invalidate_pair(FL, r);
    p.m.flags |= DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST;
    return;
  }
  // no NAT state to translate with (nf.rs:143-152)
  if (f.pf == DP_PF_NONE) { p.done(DP_DONE_FILTERED); return; }
  // handle_icmp_error_port_forwarding (portfw/icmp_handling.rs:51-90): the
  // embedded packet back to its form before the state's translation
  // (nat_translate_icmp_inner, icmp_error_msg.rs:46-146), then the error
  // itself NATed by the state (nat_packet)
  Emb &em = p.h.emb;
  const Ip &a = f.pf_ip;
  if (em.net != a.fam || (f.pf == DP_PF_DST_NAT && !ip_unicast(a))) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
  const bool src = f.pf == DP_PF_DST_NAT;  // DstNat: the inner source
  uint8_t *q = em.net == 4 ? (src ? em.v4.src : em.v4.dst) : (src ? em.v6.src : em.v6.dst);
  memcpy(q, a.b, a.fam == 4 ? 4 : 16);
  uint16_t old;
  if (emb_port(em, src, old) && old != f.pf_port) emb_set_port(em, src, f.pf_port);
  if (!pf_nat_packet(p, f.pf, a, f.pf_port)) { p.done(DP_DONE_INTERNAL_FAILURE); return; }
  // is_icmp_unrecoverable (nf.rs:42-60): destination unreachable other than
  // fragmentation needed (v4), any destination unreachable (v6)
  const uint8_t t = p.h.icmp.raw[0], c = p.h.icmp.raw[1];
  const bool unrec = p.h.l4 == L4_ICMP4 ? (t == 3 && c != 4) : t == 1;
  if (unrec && FL->nfs[f.pf_status] == DP_NFS_ONE_WAY) flow_invalidate_pair(FL, r);
  p.m.flags |= DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST;  // nf.rs:176-179
}

bool adj_lookup(const dpo_tables &T, const Ip &ip, uint32_t oif, uint8_t mac[6]) {
  MacKey k{oif, ip};
  if (k.ip.fam == 4) memset(k.ip.b + 4, 0, 12);
  auto it = T.adjs.find(k);
  if (it == T.adjs.end()) return false;
  memcpy(mac, it->second.mac, 6);
  return true;
}

// Egress (dataplane/src/packet_processor/egress.rs:54-208)
void stage_egress(const dpo_tables &T, Packet &p) {
  if (p.is_done()) return;
  if (!p.m.has_oif) { p.done(DP_DONE_ROUTE_FAILURE); return; }
  uint32_t oif = p.m.oif;
  Ip nh;
  if (p.m.has_nh) nh = p.m.nh;
  else if (p.h.net) nh = ip_dst(p.h);
  else { p.done(DP_DONE_NOT_IP); return; }
  uint8_t dmac[6];
  if (!adj_lookup(T, nh, oif, dmac)) { p.done(DP_DONE_MISS_L2_RESOLUTION); return; }
  static const uint8_t zero[6] = {0};
  if (memcmp(dmac, zero, 6) == 0) { p.done(DP_DONE_INVALID_DST_MAC); return; }
  const dp_iface_t *i = find_iface(T, oif);
  if (!i) { p.done(DP_DONE_INTERFACE_UNKNOWN); return; }
  if (i->admin_state == DP_IF_DOWN) { p.done(DP_DONE_INTERFACE_ADM_DOWN); return; }
  if (i->oper_state == DP_IF_DOWN) { p.done(DP_DONE_INTERFACE_OPER_DOWN); return; }
  if (!iface_has_mac(*i)) { p.done(DP_DONE_INTERFACE_UNSUPPORTED); return; }
  if (p.h.has_eth) {
    memcpy(p.h.eth.src, i->mac, 6);
    memcpy(p.h.eth.dst, dmac, 6);
  } else {
    uint16_t et;
    if (p.h.net == 4) et = 0x0800;
    else if (p.h.net == 6) et = 0x86dd;
    else { p.done(DP_DONE_MISSING_ETHER_TYPE); return; }
    p.h.has_eth = true;
    memcpy(p.h.eth.src, i->mac, 6);
    memcpy(p.h.eth.dst, dmac, 6);
    p.h.eth.type = et;
  }
  p.done(DP_DONE_DELIVERED);
}

// Packet::serialize (net/src/packet/mod.rs:342-374)
void serialize(Packet &p) {
  update_checksums(p.h, p.buf + p.pay_start, p.pay_end - p.pay_start);
  p.m.flags &= ~DP_META_REFR_CHKSUM;
  int need = p.h.size();
  if ((int64_t)p.pay_start - need < (int64_t)p.room_start) {
    p.done_force(DP_DONE_NO_HEAD_ROOM);
    return;
  }
  deparse_headers(p.h, p.buf + p.pay_start - need);
  p.pay_start -= (uint64_t)need;
}

// The stages before FlowFilter (Packet::new .. FlowLookup); false when the
// frame is rejected (out is final then).
// The records of a packet no stage annotated.
void out_none(const dp_pkt_in_t &in, dp_pkt_out_t &out, dp_pkt_meta_t &meta, uint8_t done) {
  out = dp_pkt_out_t{};
  out.off = in.off;
  out.len = in.len;
  out.done = done;
  meta = dp_pkt_meta_t{};
  meta.fib_entry = meta.acl_rule = UINT32_MAX;
  meta.flow_ref = DP_FLOW_NONE;
}

bool process_pre(const dpo_tables &T, dpo_flows *FL, uint8_t *buf, const dp_pkt_in_t &in,
                 dp_pkt_out_t &out, dp_pkt_meta_t &meta, Packet &p) {
  p.buf = buf;
  p.room_start = in.off >= DP_HEADROOM ? in.off - DP_HEADROOM : 0;
  out_none(in, out, meta, DP_DONE_NONE);
  int c = parse_headers(buf + in.off, in.len, p.h);
  if (c < 0) {  // Packet::new fails: frame rejected by the driver (worker.rs:409-421)
    out.done = DP_DONE_NOT_ETHERNET;
    return false;
  }
  p.pay_start = in.off + (uint64_t)c;
  p.pay_end = in.off + (uint64_t)in.len;

  if (in.flags & DP_IN_SEEDED_OVERLAY) {
    // state right after IP-Forward-1's decap (ipforward.rs:140-161)
    auto it = T.vni_fib.find(in.src_vni);
    if (it == T.vni_fib.end()) p.done(DP_DONE_UNROUTABLE);
    else {
      p.m.src_vni = in.src_vni;
      p.m.has_vrf = true;
      p.m.vrf = T.fibs[it->second].d.vrf_id;
      p.m.flags |= DP_META_IS_OVERLAY;
    }
  } else {
    stage_ingress(T, p, in.iif);
    stage_ipforward(T, p);  // IP-Forward-1
  }
  stage_icmp_error(T, FL, p);
  stage_flow_lookup(FL, p);  // identity with no (or an empty) flow table
  return true;
}

// The stages after FlowFilter (AclFilter .. Egress) and serialize.
void process_post(const dpo_tables &T, dpo_flows *FL, Packet &p, dp_pkt_out_t &out, dp_pkt_meta_t &meta) {
  stage_acl(T, FL, p);
  stage_static_nat(T, p);
  stage_portfw(T, FL, p);
  stage_masquerade(T, FL, p);
  stage_ipforward(T, p);  // IP-Forward-2
  stage_egress(T, p);
  if (p.m.done == DP_DONE_DELIVERED) serialize(p);
  out.done = p.m.done < 0 ? (uint8_t)DP_DONE_NONE : (uint8_t)p.m.done;
  out.meta_flags = (uint16_t)p.m.flags;
  out.oif = p.m.has_oif ? p.m.oif : 0;
  out.acl = p.m.acl;
  // the rest of PacketMeta (net/src/packet/meta.rs:138-154)
  meta.dst_vni = p.m.dst_vni;
  meta.src_vni = p.m.src_vni;
  meta.fib_entry = p.m.fib_entry;
  meta.acl_rule = p.m.acl_rule;
  meta.pm_flags = 0;
  if (p.m.has_vrf) { meta.pm_flags |= DP_PM_HAS_VRF; meta.vrf = p.m.vrf; }
  if (p.m.has_dscp) { meta.pm_flags |= DP_PM_HAS_DSCP; meta.dscp = p.m.dscp; meta.ecn = p.m.ecn; }
  if (p.m.has_nh) {
    meta.pm_flags |= DP_PM_HAS_NH;
    meta.nh_family = p.m.nh.fam;
    memcpy(meta.nh_addr, p.m.nh.b, p.m.nh.fam == 6 ? 16 : 4);  // IpAddr: v4 is 4 bytes
  }
  meta.flow_ref = p.flow >= 0 ? (uint64_t)p.flow : DP_FLOW_NONE;
  if (p.m.done == DP_DONE_DELIVERED) {
    out.off = (uint32_t)p.pay_start;
    out.len = (uint16_t)(p.pay_end - p.pay_start);
  }
}

// Without a flow table the stages of different packets share no state, so the
// burst is processed packet by packet.
void process_one(const dpo_tables &T, uint8_t *buf, const dp_pkt_in_t &in, dp_pkt_out_t &out,
                 dp_pkt_meta_t &meta) {
  Packet p;
  if (!process_pre(T, nullptr, buf, in, out, meta, p)) return;
  FfWork w;
  ff_classify(T, nullptr, p, w);
  ff_apply(T, nullptr, p, w);
  process_post(T, nullptr, p, out, meta);
}

// With a flow table, in the reference's burst order: the lazy stages up to
// FlowLookup packet by packet, FlowFilter over the materialised burst (all
// classifications, then all route applications: flow-filter/src/lib.rs:75-111,
// 352-363), then the lazy stages after it packet by packet.
void process_burst_flows(const dpo_tables &T, dpo_flows *FL, uint8_t *buf, const dp_pkt_in_t *in,
                         dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n) {
  masq_sync(T, FL);
  FL->in_burst = true;
  std::vector<Packet> P(n);
  std::vector<char> live(n);
  std::vector<FfWork> W(n);
  for (uint32_t i = 0; i < n; i++) live[i] = process_pre(T, FL, buf, in[i], out[i], meta[i], P[i]);
  for (uint32_t i = 0; i < n; i++) if (live[i]) ff_classify(T, FL, P[i], W[i]);
  for (uint32_t i = 0; i < n; i++) if (live[i]) ff_apply(T, FL, P[i], W[i]);
  for (uint32_t i = 0; i < n; i++)
    if (live[i]) process_post(T, FL, P[i], out[i], meta[i]);
  // the flows replaced during the burst are dropped after it
  FL->in_burst = false;
  for (int64_t r : FL->departed) FL->f[r].m_alloc.reset();
  FL->departed.clear();
}

FKey fkey_of(const dp_flow_key_t &x) {
  FKey k;
  k.vni = x.src_vni; k.kind = x.kind; k.sp = x.sport; k.dp = x.dport;
  key_addrs(k, x.family == 4 ? 4 : 6, x.src, x.dst);
  if (x.family != 4 && x.family != 6) k.fam = x.family;
  return k;
}
// What a FlowInfo can hold here (dpgpu.h dp_flow_t).
int flow_check(const dp_flow_t &f) {
  const dp_flow_key_t &x = f.key;
  if (x.family != 4 && x.family != 6) return DP_EINVAL;
  if (x.kind < DP_FLOW_TCP || x.kind > DP_FLOW_ICMP_OTHER) return DP_EINVAL;
  if ((x.kind == DP_FLOW_TCP || x.kind == DP_FLOW_UDP) && (x.sport == 0 || x.dport == 0))
    return DP_EINVAL;  // TcpPort / UdpPort are non-zero
  if (x.kind == DP_FLOW_ICMP_QUERY && x.dport) return DP_EINVAL;
  if (x.kind == DP_FLOW_ICMP_OTHER && (x.sport || x.dport)) return DP_EINVAL;
  if (x.src_vni >= (1u << 24) || f.dst_vni == 0 || f.dst_vni >= (1u << 24)) return DP_EINVAL;
  if (f.flags & ~7u) return DP_EINVAL;
  return 0;
}
// FlowTable::insert_common (table.rs:215-260).  `partner`: the related flow
// of a pair (the capacity exception for the second half, :221-233).
int32_t flow_insert_one(dpo_flows *FL, const dp_flow_t &d, int64_t partner, int64_t &ref) {
  ref = -1;
  if (FL->map.size() >= FL->capacity &&
      !(partner >= 0 && FL->f[partner].status == DP_FLOW_ACTIVE))
    return DP_EFLOWCAP;
  OFlow nf;
  nf.d = d;
  nf.key = fkey_of(d.key);
  nf.status = DP_FLOW_ACTIVE;
  nf.in_table = true;
  ref = (int64_t)FL->f.size();
  int32_t res = DP_FLOW_INSERTED;
  auto it = FL->map.find(nf.key);
  if (it != FL->map.end()) {
    OFlow &old = FL->f[it->second];
    const bool was_expired = old.status == DP_FLOW_EXPIRED;
    old.status = DP_FLOW_DETACHED;
    old.in_table = false;
    flow_depart(FL, (int64_t)it->second);
    it->second = (uint64_t)ref;
    if (!was_expired) res = DP_FLOW_REPLACED;
  } else {
    FL->map.emplace(nf.key, (uint64_t)ref);
  }
  FL->f.push_back(nf);
  return res;
}
void flow_info_of(const dpo_flows *FL, int64_t r, dp_flow_info_t &o) {
  memset(&o, 0, sizeof(o));
  o.ref = DP_FLOW_NONE;
  o.related = DP_FLOW_NONE;
  if (r < 0 || !FL->f[r].in_table) return;
  const OFlow &f = FL->f[r];
  o.ref = (uint64_t)r;
  o.status = f.status;
  o.flags = f.d.flags;
  o.dst_vni = f.d.dst_vni;
  o.genid = f.d.genid;
  o.expires_at = f.d.expires_at;
  if (flow_alive(FL, f.related)) o.related = (uint64_t)f.related;
  o.pf = f.pf;
  o.masq = f.masq;
  if (f.masq != DP_PF_NONE) {  // the NAT state's fields share pf_*
    o.pf_status = FL->nfs[f.m_status];
    o.pf_port = f.m_port;
    o.pf_family = f.m_ip.fam;
    memcpy(o.pf_ip, f.m_ip.b, f.m_ip.fam == 4 ? 4 : 16);
    o.masq_alloc = f.m_alloc ? 1 : 0;
    o.idle_timeout_s = (uint32_t)(f.m_idle_ns / 1000000000ull);
  }
  if (f.pf != DP_PF_NONE) {
    o.pf_status = FL->nfs[f.pf_status];
    o.pf_port = f.pf_port;
    o.pf_rule = f.pf_rule;
    o.pf_family = f.pf_ip.fam;
    memcpy(o.pf_ip, f.pf_ip.b, f.pf_ip.fam == 4 ? 4 : 16);
  }
}

bool valid_prefix(const dp_prefix_t &p) {
  int bits = p.family == 4 ? 32 : 128;
  if (p.family != 4 && p.family != 6) return false;
  if (p.len > bits) return false;
  for (int i = p.len; i < bits; i++) if (bit_at(p.addr, i)) return false;
  return true;
}

}  // namespace

extern "C" {

int dpo_tables_build2(const dp_tables_desc_t *d, const dpo_tables_t *prev, dpo_tables_t **out) {
  if (!d || !out) return DP_EINVAL;
  auto T = std::make_unique<dpo_tables>();
  T->genid = d->genid;
  for (uint32_t i = 0; i < d->n_fibs; i++) {
    Fib f;
    f.d = d->fibs[i];
    T->fibs.push_back(std::move(f));
    T->vrf_fib[d->fibs[i].vrf_id] = i;
  }
  for (uint32_t i = 0; i < d->n_vni_fibs; i++) {
    if (d->vni_fibs[i].fib >= d->n_fibs) return DP_EINVAL;
    T->vni_fib[d->vni_fibs[i].vni] = d->vni_fibs[i].fib;
  }
  T->nhs.assign(d->route_nhs, d->route_nhs + d->n_route_nhs);
  T->entries.assign(d->entries, d->entries + d->n_entries);
  T->instrs.assign(d->instrs, d->instrs + d->n_instrs);
  for (auto &e : T->entries) {
    if (e.n_instr == 0 || e.n_instr > 4 || e.first_instr + e.n_instr > d->n_instrs) return DP_EINVAL;
    // Supported instruction forms: at most one Encap, and no Local/Encap
    // after an Encap (a re-encapsulated packet is never routed again here).
    int encaps = 0;
    for (uint32_t k = 0; k < e.n_instr; k++) {
      uint32_t kd = d->instrs[e.first_instr + k].kind;
      if (kd > DP_INSTR_EGRESS) return DP_EINVAL;
      if (encaps && (kd == DP_INSTR_LOCAL || kd == DP_INSTR_ENCAP_VXLAN)) return DP_ENOTSUP;
      if (kd == DP_INSTR_ENCAP_VXLAN) encaps++;
    }
  }
  for (auto &n : T->nhs)
    if (n.n_entries == 0 || n.first_entry + n.n_entries > d->n_entries) return DP_EINVAL;
  // Fib::default(): /0 -> drop group for v4 and v6 (routing/src/fib/fibtype.rs:76-91)
  uint32_t drop_nh = (uint32_t)T->nhs.size();
  T->instrs.push_back(dp_instr_t{DP_INSTR_DROP, 0, 0, 0, {}, {0}, {0}});
  T->entries.push_back(dp_fib_entry_t{(uint32_t)T->instrs.size() - 1, 1});
  T->nhs.push_back(dp_route_nh_t{(uint32_t)T->entries.size() - 1, 1});
  for (auto &f : T->fibs) {
    uint8_t z[16] = {0};
    f.v4.insert(z, 0, drop_nh);
    f.v6.insert(z, 0, drop_nh);
  }
  for (uint64_t i = 0; i < d->n_routes; i++) {
    const dp_route_t &r = d->routes[i];
    if (r.fib >= d->n_fibs || r.nh >= d->n_route_nhs || !valid_prefix(r.prefix)) return DP_EINVAL;
    Fib &f = T->fibs[r.fib];
    if (r.prefix.family == 4) f.v4.insert(r.prefix.addr, r.prefix.len, r.nh);
    else f.v6.insert(r.prefix.addr, r.prefix.len, r.nh);
  }
  for (uint32_t i = 0; i < d->n_ifaces; i++) T->ifaces[d->ifaces[i].ifindex] = d->ifaces[i];
  for (uint32_t i = 0; i < d->n_adjs; i++) {
    MacKey k{d->adjs[i].ifindex, Ip{}};
    k.ip.fam = d->adjs[i].addr.family;
    memcpy(k.ip.b, d->adjs[i].addr.addr, 16);
    if (k.ip.fam == 4) memset(k.ip.b + 4, 0, 12);
    T->adjs[k] = d->adjs[i];
  }
  auto load = [&](const dp_rule_t *rs, uint32_t n, std::vector<Rule> &dst, bool sort_prio) -> int {
    for (uint32_t i = 0; i < n; i++) {
      if (!valid_prefix(rs[i].src) || !valid_prefix(rs[i].dst)) return DP_EINVAL;
      dst.push_back(Rule{rs[i], i});
    }
    if (sort_prio)
      std::stable_sort(dst.begin(), dst.end(), [](const Rule &a, const Rule &b) {
        return a.r.priority > b.r.priority;
      });
    return 0;
  };
  int rc;
  if ((rc = load(d->acl_v4, d->n_acl_v4, T->acl4, false))) return rc;
  if ((rc = load(d->acl_v6, d->n_acl_v6, T->acl6, false))) return rc;
  if ((rc = load(d->ff_remote_v4, d->n_ff_remote_v4, T->ffr4, true))) return rc;
  if ((rc = load(d->ff_local_v4, d->n_ff_local_v4, T->ffl4, true))) return rc;
  if ((rc = load(d->ff_remote_v6, d->n_ff_remote_v6, T->ffr6, true))) return rc;
  if ((rc = load(d->ff_local_v6, d->n_ff_local_v6, T->ffl6, true))) return rc;
  for (auto *v : {&T->ffr4, &T->ffr6})
    for (auto &r : *v) {
      if (r.r.action2 > DP_NAT_PORT_FORWARDING) return DP_EINVAL;
      if (r.r.src.len != 0 || r.r.sport_lo != 0 || r.r.sport_hi != 65535 || r.r.gate != 0) return DP_EINVAL;
    }
  for (auto *v : {&T->ffl4, &T->ffl6})
    for (auto &r : *v) {
      if (r.r.action > DP_NAT_PORT_FORWARDING) return DP_EINVAL;
      if (r.r.gate > 1) return DP_EINVAL;
      if (r.r.dst.len != 0 || r.r.dport_lo != 0 || r.r.dport_hi != 65535) return DP_EINVAL;
    }
  for (auto *v : {&T->acl4, &T->acl6})
    for (auto &r : *v)
      if (r.r.gate != 0 || r.r.action > DP_ACL_DENY || r.r.action2 > DP_ACL_SCOPE_PACKET) return DP_EINVAL;
  for (uint32_t i = 0; i < d->n_acl_defaults; i++)
    T->acl_default[{d->acl_defaults[i].src_vni, d->acl_defaults[i].dst_vni}] = d->acl_defaults[i].action;
  for (uint32_t i = 0; i < d->n_nat_tables; i++) {
    const dp_nat_table_t &nt = d->nat_tables[i];
    NatTable *tab;
    if (nt.kind == DP_NAT_TABLE_DST) tab = &T->nat_dst[nt.src_vni];
    else tab = &T->nat_src[{nt.src_vni, nt.dst_vni}];
    if (nt.first_entry + nt.n_entries > d->n_nat_entries) return DP_EINVAL;
    for (uint32_t j = 0; j < nt.n_entries; j++) {
      const dp_nat_entry_t &e = d->nat_entries[nt.first_entry + j];
      if (e.prefix.family != 4 || !valid_prefix(e.prefix)) return DP_ENOTSUP;  // NAT44 only
      NatEntry ne;
      ne.e = e;
      if (e.first_port_range + e.n_port_ranges > d->n_nat_port_ranges) return DP_EINVAL;
      if (e.first_range + e.n_ranges > d->n_nat_ranges) return DP_EINVAL;
      ne.prs.assign(d->nat_port_ranges + e.first_port_range, d->nat_port_ranges + e.first_port_range + e.n_port_ranges);
      ne.ranges.assign(d->nat_ranges + e.first_range, d->nat_ranges + e.first_range + e.n_ranges);
      // IpPortPrefixTrie::insert: a later insert of the same prefix replaces
      bool replaced = false;
      for (auto &x : tab->entries)
        if (x.e.prefix.len == e.prefix.len && memcmp(x.e.prefix.addr, e.prefix.addr, 4) == 0) {
          x = ne; replaced = true; break;
        }
      if (!replaced) tab->entries.push_back(std::move(ne));
    }
  }
  for (uint32_t i = 0; i < d->n_portfw; i++) {
    const dp_portfw_rule_t &r = d->portfw[i];
    if (!pf_valid(r) || !valid_prefix(r.ext_prefix) || !valid_prefix(r.int_prefix)) return DP_EINVAL;
  }
  pf_update(*T, prev, d->portfw, d->n_portfw);
  // masquerade exposes: one family each, a non-empty public range
  // (ValidatedExpose), and the configuration's canonical bytes
  if (d->n_masq && (!d->masq || !d->masq_prefixes)) return DP_EINVAL;
  auto put = [&](const void *x, size_t k) { T->masq_cfg.append(static_cast<const char *>(x), k); };
  for (uint32_t i = 0; i < d->n_masq; i++) {
    const dp_masq_expose_t &x = d->masq[i];
    if (!x.src_vni || !x.dst_vni || x.src_vni == x.dst_vni || !x.n_public || !x.n_private) return DP_EINVAL;
    if ((uint64_t)x.first_prefix + x.n_private + x.n_public > d->n_masq_prefixes) return DP_EINVAL;
    if ((uint64_t)x.first_claim + x.n_claims > d->n_masq_claims) return DP_EINVAL;
    MExpose e;
    e.src_vni = x.src_vni;
    e.dst_vni = x.dst_vni;
    e.idle_ns = (uint64_t)(x.idle_timeout_s ? x.idle_timeout_s : 120) * 1000000000ull;
    e.fam = d->masq_prefixes[x.first_prefix].family;
    for (uint32_t k = 0; k < (uint32_t)x.n_private + x.n_public; k++) {
      const dp_prefix_t &q = d->masq_prefixes[x.first_prefix + k];
      if (!valid_prefix(q) || q.family != e.fam) return DP_EINVAL;
      (k < x.n_private ? e.priv : e.pub).push_back(q);
    }
    for (uint32_t k = 0; k < x.n_claims; k++) {
      const dp_masq_claim_t &c = d->masq_claims[x.first_claim + k];
      if (!valid_prefix(c.prefix) || c.lo > c.hi) return DP_EINVAL;
      e.claims.push_back(c);
    }
    put(&x.src_vni, 4); put(&x.dst_vni, 4); put(&e.idle_ns, 8);
    for (auto *v : {&e.priv, &e.pub}) {
      const uint32_t m = (uint32_t)v->size();
      put(&m, 4);
      for (auto &q : *v) put(&q, sizeof q);
    }
    const uint32_t m = (uint32_t)e.claims.size();
    put(&m, 4);
    for (auto &c : e.claims) put(&c, sizeof c);
    T->masq.push_back(std::move(e));
  }
  T->masq_tag = d->masq_config_tag;
  T->masq_random = d->masq_randomize != 0;
  T->masq_seed = d->masq_seed;
  static std::atomic<uint64_t> serials{1};
  T->serial = serials++;
  *out = T.release();
  return 0;
}

int dpo_tables_build(const dp_tables_desc_t *d, dpo_tables_t **out) { return dpo_tables_build2(d, nullptr, out); }

int dpo_flows_sync(dpo_flows_t *fl, const dpo_tables_t *t) {
  if (!fl || !t) return DP_EINVAL;
  masq_sync(*t, fl);
  return 0;
}

int dpo_flows_set_clock(dpo_flows_t *fl, uint64_t now) {
  if (!fl) return DP_EINVAL;
  fl->now = now;
  return 0;
}
int dpo_portfw_rule_alive(const dpo_tables_t *t, uint32_t id) { return t && pf_by_id(*t, id) ? 1 : 0; }

void dpo_tables_free(dpo_tables_t *t) { delete t; }

int dpo_process_burst(const dpo_tables_t *t, uint8_t *buf, uint64_t buf_bytes,
                      const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n,
                      uint64_t *stats) {
  if (!t || (!buf && n) || (!out && n)) return DP_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    if (in[i].off < DP_HEADROOM || (uint64_t)in[i].off + in[i].len > buf_bytes) return DP_EINVAL;
  }
  for (uint32_t i = 0; i < n; i++) {
    dp_pkt_meta_t m;
    process_one(*t, buf, in[i], out[i], meta ? meta[i] : m);
    if (stats && out[i].done < DP_DONE_COUNT) stats[out[i].done]++;
  }
  return 0;
}

int dpo_process_parallel(const dpo_tables_t *t, uint8_t *buf, uint64_t buf_bytes,
                         const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n,
                         uint32_t burst, uint32_t threads) {
  if (!t || threads == 0 || burst == 0) return DP_EINVAL;
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < threads; k++) {
    th.emplace_back([&]() {
      for (;;) {
        uint32_t s = next.fetch_add(burst);
        if (s >= n) break;
        uint32_t e = std::min(n, s + burst);
        dpo_process_burst(t, buf, buf_bytes, in + s, out + s, meta ? meta + s : nullptr, e - s, nullptr);
      }
    });
  }
  for (auto &x : th) x.join();
  return 0;
}

int dpo_process_burst_flows(const dpo_tables_t *t, dpo_flows_t *fl, uint8_t *buf, uint64_t buf_bytes,
                            const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n,
                            uint64_t *stats) {
  if (!t || (!buf && n) || ((!out || !meta) && n)) return DP_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (in[i].off < DP_HEADROOM || (uint64_t)in[i].off + in[i].len > buf_bytes) return DP_EINVAL;
  if (!fl) {
    for (uint32_t i = 0; i < n; i++) process_one(*t, buf, in[i], out[i], meta[i]);
  } else {
    process_burst_flows(*t, fl, buf, in, out, meta, n);
  }
  if (stats)
    for (uint32_t i = 0; i < n; i++) if (out[i].done < DP_DONE_COUNT) stats[out[i].done]++;
  return 0;
}

int dpo_flows_create(dpo_flows_t **out) {
  if (!out) return DP_EINVAL;
  *out = new dpo_flows();
  return 0;
}
void dpo_flows_free(dpo_flows_t *fl) { delete fl; }
int dpo_flows_set_capacity(dpo_flows_t *fl, uint64_t capacity) {
  if (!fl) return DP_EINVAL;
  fl->capacity = capacity;
  return 0;
}
int dpo_flow_insert(dpo_flows_t *fl, const dp_flow_t *flows, uint32_t n, uint64_t *refs,
                    int32_t *results) {
  if (!fl || (!flows && n)) return DP_EINVAL;
  for (uint32_t i = 0; i < n; i++) if (int rc = flow_check(flows[i])) return rc;
  for (uint32_t i = 0; i < n; i++) {
    int64_t r;
    const int32_t res = flow_insert_one(fl, flows[i], -1, r);
    if (refs) refs[i] = r < 0 ? DP_FLOW_NONE : (uint64_t)r;
    if (results) results[i] = res;
  }
  return 0;
}
// FlowInfo::related_pair (flow_info.rs:290-339), then both inserts
int dpo_flow_insert_pair(dpo_flows_t *fl, const dp_flow_t *a, const dp_flow_t *b, uint64_t *refs,
                         int32_t *results) {
  if (!fl || !a || !b) return DP_EINVAL;
  if (int rc = flow_check(*a)) return rc;
  if (int rc = flow_check(*b)) return rc;
  if (fkey_of(a->key) == fkey_of(b->key)) return DP_EINVAL;
  if (((a->flags ^ b->flags) & DP_FLOW_INITIATOR) == 0) return DP_EINVAL;
  int64_t ra, rb;
  const int32_t res_a = flow_insert_one(fl, *a, -1, ra);
  const int32_t res_b = flow_insert_one(fl, *b, ra, rb);
  if (ra >= 0 && rb >= 0) { fl->f[ra].related = rb; fl->f[rb].related = ra; }
  if (refs) {
    refs[0] = ra < 0 ? DP_FLOW_NONE : (uint64_t)ra;
    refs[1] = rb < 0 ? DP_FLOW_NONE : (uint64_t)rb;
  }
  if (results) { results[0] = res_a; results[1] = res_b; }
  return 0;
}
int dpo_flow_lookup(dpo_flows_t *fl, const dp_flow_key_t *keys, uint32_t n, dp_flow_info_t *out) {
  if (!fl || ((!keys || !out) && n)) return DP_EINVAL;
  for (uint32_t i = 0; i < n; i++) flow_info_of(fl, flow_find(fl, fkey_of(keys[i])), out[i]);
  return 0;
}
int dpo_flow_get(dpo_flows_t *fl, const uint64_t *refs, uint32_t n, dp_flow_info_t *out) {
  if (!fl || ((!refs || !out) && n)) return DP_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    flow_info_of(fl, refs[i] < fl->f.size() ? (int64_t)refs[i] : -1, out[i]);
  return 0;
}
int dpo_flow_remove(dpo_flows_t *fl, const dp_flow_key_t *keys, uint32_t n, uint32_t *n_removed) {
  if (!fl || (!keys && n)) return DP_EINVAL;
  uint32_t c = 0;
  for (uint32_t i = 0; i < n; i++) {
    auto it = fl->map.find(fkey_of(keys[i]));
    if (it == fl->map.end()) continue;
    OFlow &f = fl->f[it->second];
    f.status = DP_FLOW_DETACHED;
    f.in_table = false;
    flow_depart(fl, (int64_t)it->second);
    fl->map.erase(it);
    c++;
  }
  if (n_removed) *n_removed = c;
  return 0;
}
int dpo_flow_invalidate(dpo_flows_t *fl, const uint64_t *refs, uint32_t n) {
  if (!fl || (!refs && n)) return DP_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    if (refs[i] < fl->f.size() && fl->f[refs[i]].in_table) flow_invalidate_pair(fl, (int64_t)refs[i]);
  return 0;
}
int dpo_flow_set_status(dpo_flows_t *fl, uint64_t ref, uint32_t status) {
  if (!fl || status > DP_FLOW_DETACHED) return DP_EINVAL;
  if (ref >= fl->f.size() || !fl->f[ref].in_table) return DP_EINVAL;
  fl->f[ref].status = status;
  return 0;
}
// The flow timers up to `now` (table.rs:160-213)
int dpo_flow_sweep(dpo_flows_t *fl, uint64_t now, uint64_t *n_removed) {
  if (!fl) return DP_EINVAL;
  uint64_t c = 0;
  for (auto it = fl->map.begin(); it != fl->map.end();) {
    OFlow &f = fl->f[it->second];
    bool gone = false;
    if (f.status == DP_FLOW_ACTIVE) {
      if (f.d.expires_at <= now) { f.status = DP_FLOW_EXPIRED; gone = true; }
    } else if (f.status == DP_FLOW_CANCELLED || f.status == DP_FLOW_EXPIRED) {
      gone = true;
    }
    if (gone) { f.in_table = false; flow_depart(fl, (int64_t)it->second); it = fl->map.erase(it); c++; }
    else ++it;
  }
  if (n_removed) *n_removed = c;
  return 0;
}
int dpo_flow_count(dpo_flows_t *fl, uint64_t *len, uint64_t *active) {
  if (!fl) return DP_EINVAL;
  uint64_t a = 0;
  for (auto &kv : fl->map) a += fl->f[kv.second].status == DP_FLOW_ACTIVE;
  if (len) *len = fl->map.size();
  if (active) *active = a;
  return 0;
}

uint16_t dpo_checksum_ipv4_header(const uint8_t *hdr, uint32_t hlen) {
  uint8_t tmp[60];
  memcpy(tmp, hdr, hlen);
  tmp[10] = tmp[11] = 0;
  Sum16 s;
  s.add_slice(tmp, hlen);
  return s.ones_complement();
}

int64_t dpo_lpm(const dpo_tables_t *t, uint32_t fib, uint8_t family, const uint8_t *addr) {
  if (!t || fib >= t->fibs.size()) return -1;
  Ip a;
  a.fam = family;
  memcpy(a.b, addr, family == 4 ? 4 : 16);
  return fib_lpm(t->fibs[fib], a);
}

int64_t dpo_acl_lookup(const dpo_tables_t *t, uint8_t family, uint8_t proto, uint32_t src_vni,
                       uint32_t dst_vni, const uint8_t *src, const uint8_t *dst, int has_ports,
                       uint16_t sport, uint16_t dport) {
  Key k{proto, src_vni, dst_vni, 0, src, dst, (uint16_t)(has_ports ? sport : 0),
        (uint16_t)(has_ports ? dport : 0)};
  const auto &tab = family == 4 ? t->acl4 : t->acl6;
  int64_t r = classify(tab, k, family);
  return r < 0 ? -1 : (int64_t)tab[r].orig_index;
}

// The ACL classifier alone (dpgpu.h dp_acl_classify): AclFilter's decision
// for a key (acl-filter/src/lib.rs:96-137): the first matching rule of the
// peering, else its default, else Allow.
int dpo_acl_classify(const dpo_tables_t *t, const dp_acl_key_t *keys, dp_acl_result_t *out, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    const dp_acl_key_t &k = keys[i];
    dp_acl_result_t r{};
    r.rule = UINT32_MAX;
    if (k.family == 4 || k.family == 6) {
      const Key key{k.proto, k.src_vni, k.dst_vni, 0, k.src, k.dst, k.sport, k.dport};
      const auto &tab = k.family == 4 ? t->acl4 : t->acl6;
      const int64_t ri = classify(tab, key, k.family);
      if (ri >= 0) {
        r.rule = tab[ri].orig_index;
        r.action = (uint8_t)tab[ri].r.action;
        r.scope = (uint8_t)tab[ri].r.action2;
        r.acl = r.action == DP_ACL_DENY ? 2 : 1;
      } else {
        auto it = t->acl_default.find({k.src_vni, k.dst_vni});
        if (it != t->acl_default.end()) {
          r.action = (uint8_t)it->second;
          r.acl = r.action == DP_ACL_DENY ? 4 : 3;
        } else {
          r.action = DP_ACL_ALLOW;
          r.acl = 5;
        }
      }
    }
    out[i] = r;
  }
  return 0;
}

// The flow-filter classifier alone (dpgpu.h dp_ff_classify):
// FlowFilterContext::lookup_batch (flow-filter/src/context/tables.rs:800-848,
// lookup_versioned :854-915) -- per input, the remote rules in priority order
// over (proto, src VNI, GateVni, destination, destination port), then on a
// hit the local rules over (proto, src VNI, the verdict's VPC, source, source
// port, SourceGate); addresses of different families: DestinationMiss.
// stage: 0 both, 1 the remote rules alone, 2 the local rules alone (dst_vni
// is then the local key's VPC), as dp_ff_classify_match runs them.
int dpo_ff_classify(const dpo_tables_t *t, const dp_ff_input_t *in, dp_ff_result_t *out, uint32_t n, int stage) {
  static const uint8_t zero16[16] = {0};
  for (uint32_t i = 0; i < n; i++) {
    const dp_ff_input_t &q = in[i];
    dp_ff_result_t r{};
    r.outcome = stage == 2 ? DP_FF_SOURCE_MISS : DP_FF_DESTINATION_MISS;
    out[i] = r;
    if (q.src_family != q.dst_family || (q.src_family != 4 && q.src_family != 6)) continue;
    const int fam = q.src_family;
    const auto &rem = fam == 4 ? t->ffr4 : t->ffr6;
    const auto &loc = fam == 4 ? t->ffl4 : t->ffl6;
    uint32_t dvni = q.dst_vni;
    if (stage != 2) {
      const Key k{q.proto, q.src_vni, q.dst_vni, 0, zero16, q.dst, 0, q.dport};
      const int64_t ri = classify(rem, k, fam);
      if (ri < 0) continue;
      r.dst_vni = rem[ri].r.action;
      r.dst_nat = (uint8_t)rem[ri].r.action2;
      dvni = r.dst_vni;
      r.outcome = stage == 1 ? DP_FF_ROUTE : DP_FF_SOURCE_MISS;
      out[i] = r;
      if (stage == 1) continue;
    }
    const Key k2{q.proto, q.src_vni, dvni, q.gate, q.src, zero16, q.sport, 0};
    const int64_t li = classify(loc, k2, fam);
    if (li < 0) continue;
    r.src_nat = (uint8_t)loc[li].r.action;
    r.outcome = DP_FF_ROUTE;
    out[i] = r;
  }
  return 0;
}

int dpo_nat_lookup(const dpo_tables_t *t, uint32_t kind, uint32_t src_vni, uint32_t dst_vni,
                   const uint8_t *addr4, int has_port, uint16_t port, uint8_t *new_addr4,
                   uint16_t *new_port) {
  const NatTable *tab = nullptr;
  if (kind == 0) {
    auto it = t->nat_dst.find(src_vni);
    if (it != t->nat_dst.end()) tab = &it->second;
  } else {
    auto it = t->nat_src.find({src_vni, dst_vni});
    if (it != t->nat_src.end()) tab = &it->second;
  }
  if (!tab) return 0;
  uint32_t na; bool hp; uint16_t np = 0;
  if (!nat_find_mapping(*tab, addr4, has_port != 0, port, na, hp, np)) return 0;
  if (kind == 1 && ((na >> 28) == 0xe || na == 0xffffffffu)) return 0;
  put32(new_addr4, na);
  *new_port = hp ? np : 0;
  return 1;
}

uint64_t dpo_hash_bytes(const uint8_t *p, uint32_t len) { return rapid(p, len); }

// Packet::new then Packet::serialize of a frame with no stage in between
// (the driver's tx of a packet built from an output frame, worker.rs:577):
// `out` receives the frame the reference would transmit.  Returns its
// length, or -1 if the frame does not parse (or exceeds `cap`).
int dpo_reserialize(const uint8_t *frame, uint32_t len, uint8_t *out, uint32_t cap) {
  Headers h;
  int c = parse_headers(frame, len, h);
  if (c < 0) return -1;
  update_checksums(h, frame + c, len - (uint32_t)c);
  const int hs = h.size();
  if ((uint32_t)hs + (len - (uint32_t)c) > cap) return -1;
  deparse_headers(h, out);
  memcpy(out + hs, frame + c, len - (uint32_t)c);
  return hs + (int)(len - (uint32_t)c);
}

}  // extern "C"

// SPDX-License-Identifier: Apache-2.0
//
// Host table compiler: lowers the dp_tables_desc_t arrays (include/dpgpu.h)
// into the device table image (dp_device.h).  Runs on the publishing
// (mgmt) thread; the result is uploaded once per generation.
//
// Semantics preserved from the reference builders:
//  - Fib::default() installs /0 -> drop for v4 and v6 unless a /0 route is
//    given (routing/src/fib/fibtype.rs:76-91); inserting a prefix twice keeps
//    the last value (PrefixMap::insert).
//  - Flow-filter tables match in stable descending-priority order
//    (flow-filter/src/context/tables.rs:373-380); ACL tables in array order
//    (acl-filter/src/context.rs:447-452).
//  - NAT tables: IpPortPrefixTrie keyed by prefix, last insert wins
//    (nat/src/static_nat/setup/mod.rs:73-95).
#include "dp_tables.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <cstddef>
#include <functional>
#include <map>
#include <set>
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#ifndef DP_V6_WTB
#define DP_V6_WTB 20  // v6 window table bits (16: 256 KiB per FIB, 20: 4 MiB)
#endif
#ifndef DP_SMALL_DBITS
#define DP_SMALL_DBITS 20  // direct-table bits of small v4 FIBs with long routes (16: off)
#endif

namespace dpd {
namespace {

typedef unsigned __int128 u128;

struct ImgBuf {
  std::vector<uint8_t> b;
  uint64_t alloc(uint64_t n, uint64_t align = 16) {
    uint64_t o = (b.size() + align - 1) & ~(align - 1);
    b.resize(o + (n ? n : align), 0);
    return o;
  }
  template <class T> uint64_t put(const std::vector<T> &v, uint64_t align = 16) {
    uint64_t o = alloc(sizeof(T) * v.size(), alignof(T) > align ? alignof(T) : align);
    if (!v.empty()) memcpy(b.data() + o, v.data(), sizeof(T) * v.size());
    return o;
  }
};

inline uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
inline bool bit_at(const uint8_t *a, int i) { return (a[i >> 3] >> (7 - (i & 7))) & 1; }

bool valid_prefix(const dp_prefix_t &p) {
  if (p.family != 4 && p.family != 6) return false;
  int bits = p.family == 4 ? 32 : 128;
  if (p.len > bits) return false;
  for (int i = p.len; i < bits; i++)
    if (bit_at(p.addr, i)) return false;
  return true;
}

// 128-bit key, MSB-aligned (bit 0 of the address is the top bit)
u128 key128(uint8_t fam, const uint8_t *a) {
  u128 k = 0;
  int n = fam == 4 ? 4 : 16;
  for (int i = 0; i < n; i++) k = (k << 8) | a[i];
  if (fam == 4) k <<= 96;
  return k;
}

// ------------------------------------------------------------------ hashing
struct KV { uint32_t k0, k1, k2, v; };

HashMap build_hash(ImgBuf &ib, const std::vector<KV> &kv) {
  HashMap m{};
  if (kv.empty()) { m.slots = ib.alloc(sizeof(HashSlot)); m.mask = 0; m.count = 0; return m; }
  uint32_t cap = 2;
  while (cap < 2 * kv.size()) cap <<= 1;
  std::vector<HashSlot> s(cap);
  memset(s.data(), 0, sizeof(HashSlot) * cap);
  uint32_t count = 0;
  for (auto &e : kv) {
    uint32_t i = hmix(e.k0, e.k1, e.k2) & (cap - 1);
    uint32_t key2 = e.k2 | 0x80000000u;
    for (;;) {
      if (!(s[i].k2 & 0x80000000u)) { s[i] = HashSlot{e.k0, e.k1, key2, e.v}; count++; break; }
      if (s[i].k0 == e.k0 && s[i].k1 == e.k1 && s[i].k2 == key2) { s[i].val = e.v; break; }
      i = (i + 1) & (cap - 1);
    }
  }
  m.slots = ib.put(s);
  m.mask = cap - 1;
  m.count = count;
  return m;
}

// ------------------------------------------------------------------ poptrie
struct PRoute { u128 key; int len; uint32_t nh; };

inline uint32_t kbits(u128 k, int off, int nb) {
  if (off >= 128) return 0;
  return (uint32_t)((k << off) >> (128 - nb));
}

struct PtBuilder {
  std::vector<PtNode> nodes;
  std::vector<uint32_t> leaves;

  void build_node(uint32_t idx, const PRoute *r, size_t n, uint32_t d, int off) {
    uint32_t slot[64];
    for (int v = 0; v < 64; v++) slot[v] = d;
    std::vector<const PRoute *> shortr;
    for (size_t i = 0; i < n; i++)
      if (r[i].len <= off + 6) shortr.push_back(&r[i]);
    std::stable_sort(shortr.begin(), shortr.end(),
                     [](const PRoute *a, const PRoute *b) { return a->len < b->len; });
    for (auto *p : shortr) {
      int L = p->len - off;  // 1..6
      uint32_t v0 = kbits(p->key, off, 6) & ~((1u << (6 - L)) - 1);
      for (uint32_t v = v0; v < v0 + (1u << (6 - L)); v++) slot[v] = p->nh;
    }
    uint64_t vec = 0;
    // long routes grouped by slot (r sorted by key -> contiguous)
    size_t gbeg[64], gend[64];
    for (int v = 0; v < 64; v++) gbeg[v] = gend[v] = 0;
    for (size_t i = 0; i < n; i++) {
      if (r[i].len <= off + 6) continue;
      uint32_t v = kbits(r[i].key, off, 6);
      if (!(vec & (1ull << v))) { vec |= 1ull << v; gbeg[v] = i; }
      gend[v] = i + 1;
    }
    uint32_t nchild = (uint32_t)__builtin_popcountll(vec);
    uint32_t base1 = (uint32_t)nodes.size();
    nodes.resize(nodes.size() + nchild);
    uint32_t base0 = (uint32_t)leaves.size();
    uint64_t leafvec = 0;
    bool first = true;
    uint32_t prev = 0;
    for (int v = 0; v < 64; v++) {
      if (vec & (1ull << v)) continue;
      if (first || slot[v] != prev) {
        leafvec |= 1ull << v;
        leaves.push_back(slot[v]);
        prev = slot[v];
        first = false;
      }
    }
    nodes[idx] = PtNode{vec, leafvec, base1, base0, 0};
    uint32_t k = 0;
    for (int v = 0; v < 64; v++) {
      if (!(vec & (1ull << v))) continue;
      // routes in [gbeg, gend) with len > off+6 (short ones may interleave)
      std::vector<PRoute> sub;
      for (size_t i = gbeg[v]; i < gend[v]; i++)
        if (r[i].len > off + 6) sub.push_back(r[i]);
      build_node(base1 + k, sub.data(), sub.size(), slot[v], off + 6);
      k++;
    }
  }
};

// v6 window (Lpm.wtab): the routes longer than the 16-bit direct table share
// their top bits (a site's or provider's prefix, e.g. 2001:db8::/32); keys
// inside that prefix read a table over the next wtb bits (`wtb_max`: DP_V6_WTB,
// 20: 4 MiB, while every FIB's window fits a 256 MiB budget over the image,
// else 16; 16 also when the prefix is longer than 64 - 20) -- the best route of length
// <= wbits + wtb, or a Poptrie node for the longer ones -- instead of walking
// the Poptrie levels down to it.  `uniq` is sorted by (key, length).
void add_v6_window(ImgBuf &ib, PtBuilder &pb, const std::vector<PRoute> &uniq, Lpm &L, int wtb_max) {
  if (wtb_max <= 0) return;
  bool any = false;
  u128 lo = 0, hi = 0;
  int minlen = 129;
  for (const PRoute &r : uniq) {
    if (r.len <= 16) continue;
    if (!any) lo = r.key;
    hi = r.key;
    any = true;
    minlen = std::min(minlen, r.len);
  }
  if (!any) return;
  const u128 x = lo ^ hi;
  int c = x == 0 ? 128 : ((uint64_t)(x >> 64) ? __builtin_clzll((uint64_t)(x >> 64)) : 64 + __builtin_clzll((uint64_t)x));
  c = std::min({c, minlen, 48});
  if (c < 24) return;
  const int wb = c + wtb_max <= 64 ? wtb_max : 16;  // window table bits
  const int sh = 128 - c;
  const u128 P = lo >> sh, base = P << sh;
  // the longest route of length <= c covering the window (the /0 at least)
  uint32_t d = 0;
  int dl = -1;
  for (const PRoute &r : uniq)
    if (r.len <= c && r.len > dl && (r.len == 0 || (r.key >> (128 - r.len)) == (base >> (128 - r.len)))) {
      d = r.nh;
      dl = r.len;
    }
  std::vector<uint32_t> val((size_t)1 << wb, d);
  std::vector<const PRoute *> mid;
  for (const PRoute &r : uniq)
    if (r.len > c && r.len <= c + wb) mid.push_back(&r);
  std::stable_sort(mid.begin(), mid.end(), [](const PRoute *a, const PRoute *b) { return a->len < b->len; });
  for (const PRoute *p : mid) {
    const uint32_t span = 1u << (c + wb - p->len);
    const uint32_t v0 = kbits(p->key, c, wb) & ~(span - 1);
    std::fill(val.begin() + v0, val.begin() + v0 + span, p->nh);
  }
  std::vector<uint32_t> tab((size_t)1 << wb);
  for (size_t k = 0; k < tab.size(); k++) tab[k] = 0x80000000u | val[k];
  size_t i = 0;
  while (i < uniq.size()) {
    if (uniq[i].len <= c + wb) { i++; continue; }
    const uint32_t slot = kbits(uniq[i].key, c, wb);
    std::vector<PRoute> sub;
    size_t j = i;
    while (j < uniq.size() && (uniq[j].key >> sh) == P && kbits(uniq[j].key, c, wb) == slot) {
      if (uniq[j].len > c + wb) sub.push_back(uniq[j]);
      j++;
    }
    const uint32_t idx = (uint32_t)pb.nodes.size();
    pb.nodes.emplace_back();
    pb.build_node(idx, sub.data(), sub.size(), val[slot], c + wb);
    tab[slot] = idx;
    i = j;
  }
  L.wtab = ib.put(tab);
  L.wpfx = (uint64_t)P;
  L.wtb = (uint32_t)wb;
  L.wbits = (uint32_t)c;
}

// Build one FIB/family LPM; routes must include a /0.
Lpm build_lpm(ImgBuf &ib, PtBuilder &pb, std::vector<PRoute> &routes, int width, uint32_t dbits, int v6wtb = 0) {
  // sort by (key, len), keep the last insert of a duplicate prefix
  std::stable_sort(routes.begin(), routes.end(), [](const PRoute &a, const PRoute &b) {
    if (a.key != b.key) return a.key < b.key;
    return a.len < b.len;
  });
  std::vector<PRoute> uniq;
  for (size_t i = 0; i < routes.size(); i++) {
    if (!uniq.empty() && uniq.back().key == routes[i].key && uniq.back().len == routes[i].len)
      uniq.back() = routes[i];
    else
      uniq.push_back(routes[i]);
  }
  std::vector<uint32_t> direct((size_t)1 << dbits, 0);
  std::vector<uint32_t> dval((size_t)1 << dbits, 0);
  // paint short routes in increasing length
  std::vector<const PRoute *> shortr;
  for (auto &r : uniq)
    if (r.len <= (int)dbits) shortr.push_back(&r);
  std::stable_sort(shortr.begin(), shortr.end(),
                   [](const PRoute *a, const PRoute *b) { return a->len < b->len; });
  for (auto *p : shortr) {
    uint64_t s0 = kbits(p->key, 0, dbits) & ~(((uint64_t)1 << (dbits - p->len)) - 1);
    uint64_t cnt = (uint64_t)1 << (dbits - p->len);
    std::fill(dval.begin() + s0, dval.begin() + s0 + cnt, p->nh);
  }
  for (size_t s = 0; s < dval.size(); s++) direct[s] = 0x80000000u | dval[s];
  Lpm L{};
  // v4 with a 24-bit direct table: DIR-24-8, one uint16_t[256] block of
  // next hops per /24 that holds longer routes -- a lookup is at most two
  // dependent loads (a Poptrie node walk below the direct table is up to
  // three: node, node, leaf).  Needs every next hop to fit in 16 bits.
  uint32_t max_nh = 0;
  for (auto &r : uniq) max_nh = std::max(max_nh, r.nh);
#ifdef DP_NO_DIR248
  max_nh = 0xffffu;
#endif
  if (width == 32 && dbits == 24 && max_nh < 0xffffu) {
    std::vector<uint16_t> blocks;
    size_t i = 0;
    while (i < uniq.size()) {
      if (uniq[i].len <= 24) { i++; continue; }
      const uint32_t s = kbits(uniq[i].key, 0, 24);
      std::vector<const PRoute *> sub;
      size_t j = i;
      while (j < uniq.size() && kbits(uniq[j].key, 0, 24) == s) {
        if (uniq[j].len > 24) sub.push_back(&uniq[j]);
        j++;
      }
      std::stable_sort(sub.begin(), sub.end(), [](const PRoute *a, const PRoute *b) { return a->len < b->len; });
      const size_t base = blocks.size();
      blocks.resize(base + 256, (uint16_t)dval[s]);
      for (auto *p : sub) {
        const uint32_t v0 = kbits(p->key, 24, 8) & ~((1u << (32 - p->len)) - 1);
        std::fill(blocks.begin() + base + v0, blocks.begin() + base + v0 + (1u << (32 - p->len)), (uint16_t)p->nh);
      }
      direct[s] = (uint32_t)(base >> 8);
      i = j;
    }
    if (blocks.empty()) blocks.resize(256, 0);
    L.blocks = ib.put(blocks);
    L.dbits = dbits;
    L.width = (uint32_t)width;
#ifdef DP_DIR16
    // 16-bit direct entries where the next hops and the blocks fit 15 bits:
    // bit 15 = leaf (next hop), else the block -- a 32 MiB table, half the
    // lines per lookup's working set
    if (max_nh < 0x8000u && blocks.size() / 256 <= 0x8000u) {
      std::vector<uint16_t> d16(direct.size());
      for (size_t k = 0; k < direct.size(); k++)
        d16[k] = (direct[k] & 0x80000000u) ? (uint16_t)(0x8000u | (direct[k] & 0x7fffu)) : (uint16_t)direct[k];
      L.direct = ib.put(d16);
      L.dbits = dbits | DPD_LPM_D16;
      return L;
    }
#endif
    L.direct = ib.put(direct);
    return L;
  }
  // long routes: one node per direct slot
  size_t i = 0;
  while (i < uniq.size()) {
    if (uniq[i].len <= (int)dbits) { i++; continue; }
    uint32_t s = kbits(uniq[i].key, 0, dbits);
    std::vector<PRoute> sub;
    size_t j = i;
    while (j < uniq.size() && kbits(uniq[j].key, 0, dbits) == s) {
      if (uniq[j].len > (int)dbits) sub.push_back(uniq[j]);
      j++;
    }
    uint32_t idx = (uint32_t)pb.nodes.size();
    pb.nodes.emplace_back();
    pb.build_node(idx, sub.data(), sub.size(), dval[s], (int)dbits);
    direct[s] = idx;
    i = j;
  }
  L.direct = ib.put(direct);
  L.dbits = dbits;
  L.width = (uint32_t)width;
#ifndef DP_NO_V6_WINDOW
  if (width == 128) add_v6_window(ib, pb, uniq, L, v6wtb);
#endif
  return L;
}

// ------------------------------------------------------------- classifier
struct CRule { dp_rule_t r; uint32_t orig; };

struct Iv { u128 lo, hi; };  // inclusive

Iv prefix_iv(const dp_prefix_t &p, int fam) {
  int w = fam == 4 ? 32 : 128;
  u128 k = key128(fam, p.addr);
  if (fam == 4) k >>= 96;
  u128 span = p.len == w ? (u128)0 : ((w == 128 && p.len == 0) ? ~(u128)0 : (((u128)1 << (w - p.len)) - 1));
  return Iv{k, k + span};
}

// `gkv_out`: group keys -> group index; `order_out`: rules in global rule
// index order (the order of the action arrays).
// Elementary-interval index of one field: multibit table (v4 addresses,
// ports; > 16 intervals) or sorted bounds (+ 16-bit jump table).  `leaf[k]`
// (< 2^31) is the value of interval k: a bit-vector row id, or a packed
// candidate run (DPD_GROUP_LIST).
// The v6 window of this image's classifiers (Image.v6w_*), set by build_image
// before the classifiers are built: every v6 rule prefix lies inside the
// prefix of g_v6w_c bits with value g_v6w_p (0 bits: no window).
thread_local int g_v6w_c = 0;
thread_local u128 g_v6w_p = 0;

// A v6 bound in the window's key space (dp_kernel.hip v6_window_key): 0 below
// the window, all ones above it, else shifted left by the window's bits with
// bit 0 set (distinct from both).  Monotonic, so the intervals keep their order.
u128 v6_window_bound(u128 x) {
  if (!g_v6w_c) return x;
  const int sh = 128 - g_v6w_c;
  if ((x >> sh) < g_v6w_p) return 0;
  if ((x >> sh) > g_v6w_p) return ~(u128)0;
  return (x << g_v6w_c) | 1;
}

void build_field_index(ImgBuf &ib, FieldIdx &F, int f, int fam, size_t ngroups,
                       const std::vector<u128> &bnd_in, const std::vector<uint32_t> &leaf) {
  // a v6 address field indexes the window's key space
  std::vector<u128> wbnd;
  if (fam == 6 && f < 2 && g_v6w_c) {
    for (const u128 &x : bnd_in) wbnd.push_back(v6_window_bound(x));
    wbnd[0] = 0;
  }
  const std::vector<u128> &bnd = wbnd.empty() ? bnd_in : wbnd;
  const size_t m = bnd.size();
  F.n = (uint32_t)m;
  F.jump = 0;
  if ((f >= 2 || fam == 4) && m > 16) {
    // multibit table over the interval partition (v4 address: 16-8-8,
    // port: 8-8; 8-8-8-8 for addresses when the table has many groups)
    const int kbits = f >= 2 ? 16 : 32;
    const int s0 = f >= 2 ? 8 : (ngroups > 128 ? 8 : 16);
    auto ivl = [&](uint64_t x) -> size_t {
      return (size_t)(std::upper_bound(bnd.begin(), bnd.end(), (u128)x) - bnd.begin()) - 1;
    };
    std::vector<uint32_t> blocks;
    std::function<uint32_t(uint64_t, int)> node = [&](uint64_t lo, int bits) -> uint32_t {
      size_t i0 = ivl(lo), i1 = ivl(lo + ((1ull << bits) - 1));
      if (i0 == i1) return DPD_LEAF | leaf[i0];
      uint32_t ch[256];
      for (uint32_t c = 0; c < 256; c++) ch[c] = node(lo + ((uint64_t)c << (bits - 8)), bits - 8);
      uint32_t bi = (uint32_t)(blocks.size() / 256);
      blocks.insert(blocks.end(), ch, ch + 256);
      return bi;
    };
    std::vector<uint32_t> root((size_t)1 << s0);
    for (uint64_t b = 0; b < root.size(); b++) root[b] = node(b << (kbits - s0), kbits - s0);
    F.root = ib.put(root);
    if (blocks.empty()) blocks.push_back(0);
    F.blocks = ib.put(blocks);
    F.s0 = (uint8_t)s0;
    F.kbits = (uint8_t)kbits;
    return;
  }
  std::vector<uint64_t> bounds;
  for (size_t k = 0; k < m; k++) {
    bounds.push_back((uint64_t)(bnd[k] >> 64));
    bounds.push_back((uint64_t)bnd[k]);
  }
  F.bounds = ib.put(bounds);
  F.rows = ib.put(leaf);
  // bucket = top 16 bits of the key: v4 address >> 16, port itself,
  // v6 address hi64 >> 48
  F.shift = f >= 2 ? 0 : (fam == 4 ? 16 : 48);
  if (m > 16) {
    std::vector<uint32_t> jump(65537);
    size_t j = 0;
    for (uint32_t b = 0; b < 65536; b++) {
      u128 start = f >= 2 ? (u128)b : (fam == 4 ? ((u128)b << 16) : ((u128)b << 112));
      while (j + 1 < m && bnd[j + 1] <= start) j++;
      jump[b] = (uint32_t)j;
    }
    jump[65536] = (uint32_t)(m - 1);
    F.jump = ib.put(jump);
  }
}

// Candidate-list limits: a group takes the list form when, for its best
// field, no interval has more than kListMax candidates and the mean list
// (over intervals) is at most kListMean; otherwise the bit-vector form.
#ifndef DP_LIST_MAX
#define DP_LIST_MAX 24
#endif
#ifndef DP_LIST_MEAN
#define DP_LIST_MEAN 6.0
#endif
constexpr uint32_t kListMax = DP_LIST_MAX;
constexpr double kListMean = DP_LIST_MEAN;

// Classifier form override for the parity tests (dpd_debug_set_classifier_form):
// 1 forces the bit-vector form, 2 takes the list form whenever the runs fit
// (<= DPD_RUN_MAX); 0 (the default): the limits above.
// forms chosen by the most recent build on this thread (test introspection)
thread_local uint32_t g_forms[2];
thread_local std::string g_group_stats;  // per-group list statistics (dpd_debug_group_stats)
thread_local std::string g_sections;     // image bytes per section (dpd_debug_image_sections)
std::atomic<int> g_cls_form{0};

int cls_form_override() { return g_cls_form.load(std::memory_order_relaxed); }

// `gkv_out`: group keys -> group index; `order_out`: rules in global rule
// index order (the order of the action arrays); `aux_patch`: image offsets
// of CandRec::aux fields with their rule (filled in once PairRecs exist).
// `kind`: 0 ACL, 1 flow-filter remote, 2 flow-filter local (which action
// words a v4 candidate record carries, CandRec4).
Classifier build_classifier(ImgBuf &ib, const std::vector<CRule> &rules, int fam, int kind,
                            std::vector<KV> *gkv_out, std::vector<const dp_rule_t *> *order_out,
                            std::vector<std::pair<uint64_t, const dp_rule_t *>> *aux_patch = nullptr) {
  Classifier C{};
  // groups in first-appearance order, rules keep their match order
  std::vector<std::vector<uint32_t>> groups;
  std::vector<KV> gkv;
  std::unordered_map<std::string, uint32_t> gidx;
  for (uint32_t i = 0; i < rules.size(); i++) {
    const dp_rule_t &r = rules[i].r;
    std::string k((const char *)&r.vni_a, 4);
    k.append((const char *)&r.vni_b, 4);
    k.push_back((char)r.gate);
    auto it = gidx.find(k);
    if (it == gidx.end()) {
      uint32_t g = (uint32_t)groups.size();
      gidx[k] = g;
      groups.emplace_back();
      gkv.push_back(KV{r.vni_a, r.vni_b, r.gate, g});
      it = gidx.find(k);
    }
    groups[it->second].push_back(i);
  }
  std::vector<uint32_t> action, action2, orig;
  std::vector<Group> grecs;
  std::vector<CandRec> recs;
  std::vector<std::pair<size_t, const dp_rule_t *>> rec_rule;  // record index -> rule (aux patch)
  for (auto &gr : groups) {
    Group G{};
    uint32_t n = (uint32_t)gr.size();
    G.n_rules = n;
    G.words = (n + 63) / 64;
    G.sum_words = (G.words + 63) / 64;
    G.rule_base = (uint32_t)action.size();
    for (uint32_t ri : gr) {
      if (order_out) order_out->push_back(&rules[ri].r);
      action.push_back(rules[ri].r.action);
      action2.push_back(rules[ri].r.action2);
      orig.push_back(rules[ri].orig);
    }
    // elementary intervals of the four fields, with the rules starting /
    // ending at each bound
    std::vector<u128> bnd[4];
    std::vector<std::vector<uint32_t>> adds[4], dels[4];
    uint32_t lmax[4];
    double lmean[4];
    for (int f = 0; f < 4; f++) {
      u128 maxv = f >= 2 ? (u128)65535 : (fam == 4 ? (u128)0xffffffffu : ~(u128)0);
      std::vector<Iv> iv(n);
      for (uint32_t j = 0; j < n; j++) {
        const dp_rule_t &r = rules[gr[j]].r;
        if (f == 0) iv[j] = prefix_iv(r.src, fam);
        else if (f == 1) iv[j] = prefix_iv(r.dst, fam);
        else if (f == 2) iv[j] = Iv{r.sport_lo, r.sport_hi};
        else iv[j] = Iv{r.dport_lo, r.dport_hi};
      }
      std::vector<u128> &b = bnd[f];
      b.push_back(0);
      for (auto &x : iv) {
        if (x.lo > x.hi) continue;  // empty range: never matches
        b.push_back(x.lo);
        if (x.hi < maxv) b.push_back(x.hi + 1);
      }
      std::sort(b.begin(), b.end());
      b.erase(std::unique(b.begin(), b.end()), b.end());
      size_t m = b.size();
      adds[f].assign(m + 1, {});
      dels[f].assign(m + 1, {});
      for (uint32_t j = 0; j < n; j++) {
        if (iv[j].lo > iv[j].hi) continue;
        size_t s = std::lower_bound(b.begin(), b.end(), iv[j].lo) - b.begin();
        size_t e = iv[j].hi < maxv ? (size_t)(std::lower_bound(b.begin(), b.end(), iv[j].hi + 1) - b.begin()) : m;
        adds[f][s].push_back(j);
        dels[f][e].push_back(j);
      }
      int64_t cnt = 0;
      uint64_t tot = 0;
      lmax[f] = 0;
      for (size_t k = 0; k < m; k++) {
        cnt += (int64_t)adds[f][k].size() - (int64_t)dels[f][k].size();
        lmax[f] = std::max(lmax[f], (uint32_t)cnt);
        tot += (uint64_t)cnt;
      }
      lmean[f] = (double)tot / (double)m;
    }
    {
      char line[256];
      snprintf(line, sizeof line, "kind %d fam %d rules %u lmax %u %u %u %u lmean %.2f %.2f %.2f %.2f\n", kind, fam, n,
               lmax[0], lmax[1], lmax[2], lmax[3], lmean[0], lmean[1], lmean[2], lmean[3]);
      g_group_stats += line;
    }
    int lf = -1;
    const int form = cls_form_override();
    for (int f = 0; f < 4 && form != 1; f++) {
      if (form == 2 ? lmax[f] > DPD_RUN_MAX : (lmax[f] > kListMax || lmean[f] > kListMean)) continue;
      if (lf < 0 || lmax[f] < lmax[lf] || (lmax[f] == lmax[lf] && lmean[f] < lmean[lf])) lf = f;
    }
    if (lf >= 0) {
      // candidate-list form: per interval of field lf, the covering rules in
      // precedence order, stored inline (identical lists shared)
      G.mode = DPD_GROUP_LIST;
      G.lfield = (uint32_t)lf;
      G.lfield2 = DPD_NO_FIELD;
      std::map<std::vector<uint32_t>, uint32_t> runs;
      // runs of field `fi`'s intervals -> index leaves
      auto list_leaves = [&](int fi, std::vector<uint32_t> &leaf) -> bool {
      std::set<uint32_t> cur;
      for (size_t k = 0; k < bnd[fi].size(); k++) {
        for (uint32_t j : dels[fi][k]) cur.erase(j);
        for (uint32_t j : adds[fi][k]) cur.insert(j);
        std::vector<uint32_t> lst(cur.begin(), cur.end());
        auto it = runs.find(lst);
        if (it == runs.end()) {
          uint32_t first = (uint32_t)recs.size();
          for (uint32_t j : lst) {
            const dp_rule_t &r = rules[gr[j]].r;
            Iv si = prefix_iv(r.src, fam), di = prefix_iv(r.dst, fam);
            CandRec c{};
            c.src_hi = (uint64_t)(si.lo >> 64); c.src_lo = (uint64_t)si.lo;
            c.dst_hi = (uint64_t)(di.lo >> 64); c.dst_lo = (uint64_t)di.lo;
            c.slen = r.src.len; c.dlen = r.dst.len;
            c.proto_val = r.proto_val; c.proto_mask = r.proto_mask;
            c.sp_lo = r.sport_lo; c.sp_hi = r.sport_hi;
            c.dp_lo = r.dport_lo; c.dp_hi = r.dport_hi;
            c.rule = G.rule_base + j;
            c.action = r.action; c.action2 = r.action2;
            c.orig = rules[gr[j]].orig;
            rec_rule.push_back({recs.size(), &r});
            recs.push_back(c);
          }
          if (recs.size() >= (1u << (31 - DPD_RUN_BITS))) return false;  // unreachable sizes
          it = runs.emplace(lst, (first << DPD_RUN_BITS) | (uint32_t)lst.size()).first;
        }
        leaf.push_back(it->second);
      }
      return true;
      };
      std::vector<uint32_t> leaf;
      if (!list_leaves(lf, leaf)) return Classifier{};
      build_field_index(ib, G.f[lf], lf, fam, groups.size(), bnd[lf], leaf);
      // v4 ACL groups: a second list index over another field whose runs fit
      // (the lookup verifies the shorter of the two runs a packet selects:
      // both hold every rule that can match it, in precedence order)
      int lf2 = -1;
#ifdef DP_TWO_ACL_INDEX
      const bool second = true;
#else
      const bool second = false;  // measured slower: off
#endif
      if (second && kind == 0 && fam == 4 && form != 2)
        for (int f = 0; f < 4; f++)
          if (f != lf && lmax[f] <= DPD_RUN_MAX && bnd[f].size() > 16 && (lf2 < 0 || lmean[f] < lmean[lf2]))
            lf2 = f;
      if (lf2 >= 0) {
        std::vector<uint32_t> leaf2;
        if (!list_leaves(lf2, leaf2)) return Classifier{};
        build_field_index(ib, G.f[lf2], lf2, fam, groups.size(), bnd[lf2], leaf2);
        G.lfield2 = (uint32_t)lf2;
      }
      grecs.push_back(G);
      g_forms[1]++;
      continue;
    }
    G.mode = DPD_GROUP_BV;
    uint32_t W = G.words, S = G.sum_words;
    std::vector<uint64_t> pool;
    std::unordered_map<std::string, uint32_t> rowid;
    auto add_row = [&](const std::vector<uint64_t> &bv) -> uint32_t {
      std::string key((const char *)bv.data(), bv.size() * 8);
      auto it = rowid.find(key);
      if (it != rowid.end()) return it->second;
      uint32_t id = (uint32_t)(pool.size() / (S + W));
      for (uint32_t s = 0; s < S; s++) {
        uint64_t m = 0;
        for (uint32_t w = s * 64; w < std::min(W, s * 64 + 64); w++)
          if (bv[w]) m |= 1ull << (w - s * 64);
        pool.push_back(m);
      }
      pool.insert(pool.end(), bv.begin(), bv.end());
      rowid[key] = id;
      return id;
    };
    // protocol (Mask predicate)
    std::vector<uint16_t> prow(256);
    for (int p = 0; p < 256; p++) {
      std::vector<uint64_t> bv(W, 0);
      for (uint32_t j = 0; j < n; j++) {
        const dp_rule_t &r = rules[gr[j]].r;
        if ((p & r.proto_mask) == (r.proto_val & r.proto_mask)) bv[j >> 6] |= 1ull << (j & 63);
      }
      prow[p] = (uint16_t)add_row(bv);
    }
    // four interval fields: bit-vector row per elementary interval
    for (int f = 0; f < 4; f++) {
      std::vector<uint64_t> cur(W, 0);
      std::vector<uint32_t> rows;
      for (size_t k = 0; k < bnd[f].size(); k++) {
        for (uint32_t j : dels[f][k]) cur[j >> 6] &= ~(1ull << (j & 63));
        for (uint32_t j : adds[f][k]) cur[j >> 6] |= 1ull << (j & 63);
        rows.push_back(add_row(cur));
      }
      build_field_index(ib, G.f[f], f, fam, groups.size(), bnd[f], rows);
    }
    G.proto_rows = ib.put(prow);
    G.pool = ib.put(pool);
    grecs.push_back(G);
    g_forms[0]++;
  }
  uint64_t recs_off;
  if (fam == 4) {
    std::vector<CandRec4> r4;
    for (const CandRec &c : recs) {
      CandRec4 x{};
      x.src = (uint32_t)c.src_lo; x.dst = (uint32_t)c.dst_lo;
      x.slen = c.slen; x.dlen = c.dlen; x.proto_val = c.proto_val; x.proto_mask = c.proto_mask;
      x.sp_lo = c.sp_lo; x.sp_hi = c.sp_hi; x.dp_lo = c.dp_lo; x.dp_hi = c.dp_hi;
      x.act0 = c.action;
      x.act1 = kind == 1 ? c.action2 : c.orig;
      x.act2 = kind == 1 ? c.aux : c.rule;
      r4.push_back(x);
    }
    recs_off = ib.put(r4, 64);
    if (aux_patch)
      for (auto &rr : rec_rule) aux_patch->push_back({recs_off + rr.first * sizeof(CandRec4) + offsetof(CandRec4, act2), rr.second});
  } else {
    recs_off = ib.put(recs, 64);
    if (aux_patch)
      for (auto &rr : rec_rule) aux_patch->push_back({recs_off + rr.first * sizeof(CandRec) + offsetof(CandRec, aux), rr.second});
  }
  for (auto &G : grecs) G.recs = recs_off;
  C.recs = recs_off;
  C.groups = build_hash(ib, gkv);
  if (gkv_out) *gkv_out = gkv;
  C.group_recs = ib.put(grecs);
  C.action = ib.put(action);
  C.action2 = ib.put(action2);
  C.orig = ib.put(orig);
  C.n_groups = (uint32_t)grecs.size();
  C.n_rules = (uint32_t)action.size();
  return C;
}

int load_rules(const dp_rule_t *rs, uint32_t n, int fam, bool by_prio, int kind,
               std::vector<CRule> &out) {
  for (uint32_t i = 0; i < n; i++) {
    const dp_rule_t &r = rs[i];
    if (!valid_prefix(r.src) || !valid_prefix(r.dst)) return DP_EINVAL;
    if (r.src.family != fam || r.dst.family != fam) return DP_EINVAL;
    if (kind == 0 && (r.gate != 0 || r.action > DP_ACL_DENY || r.action2 > DP_ACL_SCOPE_PACKET))
      return DP_EINVAL;                                                   // ACL
    if (kind == 1) {                                                      // FF remote
      if (r.src.len != 0 || r.sport_lo != 0 || r.sport_hi != 65535 || r.gate != 0) return DP_EINVAL;
      if (r.action2 > DP_NAT_PORT_FORWARDING) return DP_EINVAL;           // NatRequirement
    }
    if (kind == 2) {                                                      // FF local
      if (r.dst.len != 0 || r.dport_lo != 0 || r.dport_hi != 65535) return DP_EINVAL;
      if (r.action > DP_NAT_PORT_FORWARDING) return DP_EINVAL;
      if (r.gate > 1) return DP_EINVAL;                                   // SourceGate
    }
    out.push_back(CRule{r, i});
    // ACL: the verdict and its AclScope travel in one action word (both
    // classifier forms carry `action` to the lookup)
    if (kind == 0) out.back().r.action = r.action | (r.action2 << 8);
  }
  if (by_prio)
    std::stable_sort(out.begin(), out.end(),
                     [](const CRule &a, const CRule &b) { return a.r.priority > b.r.priority; });
  return 0;
}

// ------------------------------------------------------------ port forwarding
bool same_prefix(const dp_prefix_t &a, const dp_prefix_t &b) {
  return a.family == b.family && a.len == b.len && memcmp(a.addr, b.addr, a.family == 4 ? 4 : 16) == 0;
}
// PortFwEntry::matches (objects.rs:159-166): all but the timeouts
bool pf_matches(const dp_portfw_rule_t &a, const dp_portfw_rule_t &b) {
  return a.src_vni == b.src_vni && a.proto == b.proto && a.dst_vni == b.dst_vni &&
         same_prefix(a.ext_prefix, b.ext_prefix) && same_prefix(a.int_prefix, b.int_prefix) &&
         a.ext_lo == b.ext_lo && a.ext_hi == b.ext_hi && a.int_lo == b.int_lo && a.int_hi == b.int_hi;
}
// PortFwEntry::new's checks (objects.rs:70-155, portrange.rs:33-42)
bool pf_rule_ok(const dp_portfw_rule_t &r) {
  if (r.proto != 6 && r.proto != 17) return false;
  if (!valid_prefix(r.ext_prefix) || !valid_prefix(r.int_prefix)) return false;
  if (r.ext_prefix.family != r.int_prefix.family || r.ext_prefix.len != r.int_prefix.len) return false;
  if (!r.src_vni || !r.dst_vni || r.src_vni == r.dst_vni || r.src_vni >= (1u << 24) || r.dst_vni >= (1u << 24))
    return false;
  if (!r.ext_lo || !r.int_lo || r.ext_hi < r.ext_lo || r.int_hi < r.int_lo) return false;
  return r.ext_hi - r.ext_lo == r.int_hi - r.int_lo;
}
// PortFwTable::update (objects.rs:284-300): entries of the previous
// generation absent from the rule set go (their Weak refs die); the rules
// are added last to first (add_entry, :256-274): one matching an entry at
// its (key, prefix, port range) keeps it with the new timeouts, one whose
// range overlaps another of the same key and prefix is refused
// (RangeSet::insert_range, rangeset.rs:73-79).
PfLineage pf_update(const PfLineage &prev, const dp_portfw_rule_t *rs, uint32_t n) {
  PfLineage L;
  L.next_id = prev.next_id;
  for (const PfEntry &e : prev.live) {
    bool keep = false;
    for (uint32_t i = 0; i < n && !keep; i++) keep = pf_matches(e.r, rs[i]);
    if (keep) L.live.push_back(e);
  }
  for (uint32_t k = n; k-- > 0;) {
    const dp_portfw_rule_t &r = rs[k];
    PfEntry *exist = nullptr;
    bool overlap = false;
    for (PfEntry &e : L.live) {
      if (e.r.src_vni != r.src_vni || e.r.proto != r.proto || !same_prefix(e.r.ext_prefix, r.ext_prefix)) continue;
      if (e.r.ext_lo == r.ext_lo && e.r.ext_hi == r.ext_hi) exist = &e;
      if (e.r.ext_lo <= r.ext_hi && r.ext_lo <= e.r.ext_hi) overlap = true;
    }
    if (exist && pf_matches(exist->r, r)) {
      exist->r.init_timeout_s = r.init_timeout_s;
      exist->r.estab_timeout_s = r.estab_timeout_s;
      continue;
    }
    if (!overlap) L.live.push_back(PfEntry{r, L.next_id++});
  }
  return L;
}
void be_words(const dp_prefix_t &p, uint32_t w[4]) {
  for (int j = 0; j < 4; j++) {
    w[j] = 0;
    for (int b = 0; b < 4; b++) w[j] = (w[j] << 8) | (p.family == 4 && j > 0 ? 0 : p.addr[4 * j + b]);
  }
}

}  // namespace

int build_image(const dp_tables_desc_t *d, BuiltImage &out, PfLineage *pf) {
  g_forms[0] = g_forms[1] = 0;
  g_group_stats.clear();
  if (!d || d->abi_version != DPGPU_ABI_VERSION) return DP_EINVAL;
  ImgBuf ib;
  ib.alloc(64);  // offset 0 is never a valid structure
  g_sections.clear();
  uint64_t sec0 = ib.b.size();
  auto section = [&](const char *name) {
    g_sections += name;
    g_sections += "=" + std::to_string(ib.b.size() - sec0) + " ";
    sec0 = ib.b.size();
  };
  Image im{};
  im.genid = d->genid;

  // --- FIB objects
  for (uint32_t i = 0; i < d->n_entries; i++) {
    const dp_fib_entry_t &e = d->entries[i];
    if (e.n_instr == 0 || e.n_instr > DPD_MAX_INSTR || (uint64_t)e.first_instr + e.n_instr > d->n_instrs) return DP_EINVAL;
    int encaps = 0;
    for (uint32_t k = 0; k < e.n_instr; k++) {
      uint32_t kd = d->instrs[e.first_instr + k].kind;
      if (kd > DP_INSTR_EGRESS) return DP_EINVAL;
      if (encaps && (kd == DP_INSTR_LOCAL || kd == DP_INSTR_ENCAP_VXLAN)) return DP_ENOTSUP;
      if (kd == DP_INSTR_ENCAP_VXLAN) encaps++;
    }
    if (encaps) im.may_encap = 1;
  }
  for (uint32_t i = 0; i < d->n_route_nhs; i++) {
    const dp_route_nh_t &n = d->route_nhs[i];
    if (n.n_entries == 0 || (uint64_t)n.first_entry + n.n_entries > d->n_entries) return DP_EINVAL;
  }
  // host views of the interface and adjacency tables (last insert wins, as
  // the reference's maps do)
  std::unordered_map<uint32_t, const dp_iface_t *> ifmap;
  for (uint32_t i = 0; i < d->n_ifaces; i++) ifmap[d->ifaces[i].ifindex] = &d->ifaces[i];
  std::unordered_map<std::string, const dp_adjacency_t *> adjmap;
  auto adj_key = [](uint32_t oif, uint8_t fam, const uint8_t *addr) {
    std::string k((const char *)&oif, 4);
    k.push_back((char)fam);
    k.append((const char *)addr, fam == 6 ? 16 : 4);
    return k;
  };
  for (uint32_t i = 0; i < d->n_adjs; i++) {
    const dp_adjacency_t &a = d->adjs[i];
    if (a.addr.family != 4 && a.addr.family != 6) return DP_EINVAL;
    adjmap[adj_key(a.ifindex, a.addr.family, a.addr.addr)] = &a;
  }
  auto mac48 = [](const uint8_t *m) {
    uint64_t x = 0;
    for (int i = 0; i < 6; i++) x = (x << 8) | m[i];
    return x;
  };
  // Egress::egress_process's interface checks (egress.rs:168-190)
  auto oif_code = [&](uint32_t oif) -> uint8_t {
    auto it = ifmap.find(oif);
    if (it == ifmap.end()) return DP_DONE_INTERFACE_UNKNOWN;
    const dp_iface_t &f = *it->second;
    if (f.admin_state == DP_IF_DOWN) return DP_DONE_INTERFACE_ADM_DOWN;
    if (f.oper_state == DP_IF_DOWN) return DP_DONE_INTERFACE_OPER_DOWN;
    if (!(f.iftype == DP_IFT_ETHERNET || f.iftype == DP_IFT_DOT1Q)) return DP_DONE_INTERFACE_UNSUPPORTED;
    return 255;
  };
  std::vector<Instr> instrs;
  for (uint32_t i = 0; i < d->n_instrs; i++) {
    const dp_instr_t &s = d->instrs[i];
    Instr x{};
    x.kind = (uint8_t)s.kind;
    x.flags = (uint8_t)s.flags;
    x.fam = s.addr.family;
    x.ifindex = s.ifindex;
    x.vni = s.vni;
    memcpy(x.mac, s.mac, 6);
    memcpy(x.addr, s.addr.addr, s.addr.family == 6 ? 16 : 4);
    x.if_code = 255;
    if (s.kind == DP_INSTR_EGRESS) {
      auto it = ifmap.find(s.ifindex);
      if (it != ifmap.end()) x.eg_smac = mac48(it->second->mac);
      x.if_code = oif_code(s.ifindex);
      if (!(s.flags & DP_INSTR_HAS_IFINDEX)) {
        x.eg_code = DP_DONE_ROUTE_FAILURE;
      } else if (!(s.flags & DP_INSTR_HAS_ADDR)) {
        x.eg_code = DPD_EG_NEED_ADJ;
      } else {
        if (s.addr.family != 4 && s.addr.family != 6) return DP_EINVAL;
        auto a = adjmap.find(adj_key(s.ifindex, s.addr.family, s.addr.addr));
        if (a == adjmap.end()) x.eg_code = DP_DONE_MISS_L2_RESOLUTION;
        else if (mac48(a->second->mac) == 0) x.eg_code = DP_DONE_INVALID_DST_MAC;
        else {
          x.eg_dmac = mac48(a->second->mac);
          x.eg_code = x.if_code != 255 ? x.if_code : (uint8_t)DP_DONE_DELIVERED;
        }
      }
    }
    instrs.push_back(x);
  }
  std::vector<Entry> entries;
  for (uint32_t i = 0; i < d->n_entries; i++) entries.push_back(Entry{d->entries[i].first_instr, d->entries[i].n_instr});
  std::vector<RouteNh> nhs;
  for (uint32_t i = 0; i < d->n_route_nhs; i++) nhs.push_back(RouteNh{d->route_nhs[i].first_entry, d->route_nhs[i].n_entries});
  // default drop route object
  Instr drop{};
  drop.kind = DP_INSTR_DROP;
  instrs.push_back(drop);
  entries.push_back(Entry{(uint32_t)instrs.size() - 1, 1});
  nhs.push_back(RouteNh{(uint32_t)entries.size() - 1, 1});
  uint32_t drop_nh = (uint32_t)nhs.size() - 1;
  im.drop_nh = drop_nh;

  // routes per fib / family
  std::vector<std::vector<PRoute>> r4(d->n_fibs), r6(d->n_fibs);
  for (uint32_t f = 0; f < d->n_fibs; f++) {
    r4[f].push_back(PRoute{0, 0, drop_nh});
    r6[f].push_back(PRoute{0, 0, drop_nh});
  }
  for (uint64_t i = 0; i < d->n_routes; i++) {
    const dp_route_t &r = d->routes[i];
    if (r.fib >= d->n_fibs || r.nh >= d->n_route_nhs || !valid_prefix(r.prefix)) return DP_EINVAL;
    PRoute p{key128(r.prefix.family, r.prefix.addr), r.prefix.len, r.nh};
    (r.prefix.family == 4 ? r4 : r6)[r.fib].push_back(p);
  }
  PtBuilder pb;
  std::vector<FibRec> fibs;
  std::vector<KV> vrfkv, vnikv;
  // v4 direct tables: DIR-24-8 above 64 Ki routes; below, a 16-bit table,
  // or a 2^DP_SMALL_DBITS one for a FIB holding routes longer than /16 (host
  // routes, the VTEP /32: one Poptrie level fewer, 20 -> 26 -> leaf), while
  // those tables stay within 256 MiB over the image
  uint32_t small_long = 0;
  for (uint32_t f = 0; f < d->n_fibs; f++)
    if (r4[f].size() <= 65536)
      for (const PRoute &p : r4[f])
        if (p.len > 16) { small_long++; break; }
  const uint32_t small_d =
      (uint64_t)small_long * (4ull << DP_SMALL_DBITS) <= (256ull << 20) ? (uint32_t)DP_SMALL_DBITS : 16u;
  // v6 window tables likewise within 256 MiB over the image: 2^DP_V6_WTB
  // entries per FIB while every FIB with routes longer than /16 fits, else
  // 2^16, else none (an image with ~1000 VPC FIBs must not grow by GiB)
  uint64_t v6_long = 0;
  for (uint32_t f = 0; f < d->n_fibs; f++)
    for (const PRoute &p : r6[f])
      if (p.len > 16) { v6_long++; break; }
  const int v6wtb = v6_long * (4ull << DP_V6_WTB) <= (256ull << 20) ? DP_V6_WTB
                    : v6_long * (4ull << 16) <= (256ull << 20)      ? 16
                                                                    : 0;
  for (uint32_t f = 0; f < d->n_fibs; f++) {
    const dp_fib_t &s = d->fibs[f];
    FibRec fr{};
    fr.vrf_id = s.vrf_id;
    fr.flags = s.flags;
    fr.vtep_fam = s.vtep_ip.family;
    memcpy(fr.vtep_mac, s.vtep_mac, 6);
    memcpy(fr.vtep_ip, s.vtep_ip.addr, s.vtep_ip.family == 6 ? 16 : 4);
    uint32_t d4 = 16;
    if (r4[f].size() > 65536) d4 = 24;
    else
      for (const PRoute &p : r4[f])
        if (p.len > 16) { d4 = small_d; break; }
    fr.v4 = build_lpm(ib, pb, r4[f], 32, d4);
    fr.v6 = build_lpm(ib, pb, r6[f], 128, 16, v6wtb);
    if (fr.v6.wtab) im.v6w_fib = 1;
    fibs.push_back(fr);
    vrfkv.push_back(KV{s.vrf_id, 0, 0, f});
  }
  for (uint32_t i = 0; i < d->n_vni_fibs; i++) {
    if (d->vni_fibs[i].fib >= d->n_fibs) return DP_EINVAL;
    vnikv.push_back(KV{d->vni_fibs[i].vni, 0, 0, d->vni_fibs[i].fib});
  }
  if (pb.nodes.empty()) pb.nodes.emplace_back();
  if (pb.leaves.empty()) pb.leaves.push_back(drop_nh);
  im.pt_nodes = ib.put(pb.nodes);
  im.pt_leaves = ib.put(pb.leaves);
  im.fibs = ib.put(fibs);
  im.n_fibs = d->n_fibs;
  im.vrf_fib = build_hash(ib, vrfkv);
  std::unordered_map<uint32_t, uint32_t> vrf2fib, vni2fib;  // last insert wins
  for (auto &e : vrfkv) vrf2fib[e.k0] = e.v;
  std::vector<uint32_t> vni_order;
  for (auto &e : vnikv) {
    if (!vni2fib.count(e.k0)) vni_order.push_back(e.k0);
    vni2fib[e.k0] = e.v;
  }
  im.route_nhs = ib.put(nhs);
  im.entries = ib.put(entries);
  im.instrs = ib.put(instrs);
  // resolved next hops (one per RouteNh): a single FibEntry holding a single
  // Egress / Drop instruction is resolved in place
  std::vector<NhRec> nhrecs;
  for (const RouteNh &n : nhs) {
    NhRec r{};
    r.kind = DPD_NH_CHAIN;
    r.entry = n.first_entry;
    r.n_entries = n.n_entries;
    if (n.n_entries == 1 && entries[n.first_entry].n_instr == 1) {
      const Instr &x = instrs[entries[n.first_entry].first_instr];
      if (x.kind == DP_INSTR_EGRESS) {
        r.kind = DPD_NH_EGRESS;
        r.eg_code = x.eg_code;
        r.if_code = x.if_code;
        r.has_oif = (x.flags & DP_INSTR_HAS_IFINDEX) ? 1 : 0;
        r.oif = x.ifindex;
        r.eg_dmac = x.eg_dmac;
        r.eg_smac = x.eg_smac;
      } else if (x.kind == DP_INSTR_DROP) {
        r.kind = DPD_NH_DROP;
      }
    }
    nhrecs.push_back(r);
  }
  im.nh_recs = ib.put(nhrecs);
  im.n_nh = (uint32_t)nhrecs.size();

  section("fib");
  // --- interfaces / adjacencies
  std::vector<IfRec> ifs;
  std::vector<KV> ifkv;
  uint32_t max_if = 0;
  auto if_rec = [&](const dp_iface_t &s) {
    IfRec x{};
    x.ifindex = s.ifindex;
    x.valid = 1;
    x.pre_code = s.admin_state == DP_IF_DOWN ? (uint8_t)DP_DONE_INTERFACE_ADM_DOWN
               : !(s.iftype == DP_IFT_ETHERNET || s.iftype == DP_IFT_DOT1Q) ? (uint8_t)DP_DONE_INTERFACE_UNSUPPORTED
               : 255;
    x.post_code = s.attach == DP_ATTACH_VRF ? 255
                : s.attach == DP_ATTACH_BRIDGE ? (uint8_t)DP_DONE_INTERFACE_UNSUPPORTED
                : (uint8_t)DP_DONE_INTERFACE_DETACHED;
    x.vrf_id = s.vrf_id;
    auto f = vrf2fib.find(s.vrf_id);
    x.fib = f == vrf2fib.end() ? -1 : (int32_t)f->second;
    x.mac = mac48(s.mac);
    return x;
  };
  for (auto &kv : ifmap) {
    ifkv.push_back(KV{kv.first, 0, 0, (uint32_t)ifs.size()});
    ifs.push_back(if_rec(*kv.second));
    max_if = std::max(max_if, kv.first);
  }
  im.ifaces = build_hash(ib, ifkv);
  im.if_recs = ib.put(ifs);
  if (!ifmap.empty() && max_if < 65536) {
    std::vector<IfRec> direct(max_if + 1);
    memset(direct.data(), 0, sizeof(IfRec) * direct.size());
    for (auto &kv : ifmap) direct[kv.first] = if_rec(*kv.second);
    im.if_direct = ib.put(direct);
    im.if_direct_n = max_if + 1;
  }
  {
    uint32_t cap = 2;
    while (cap < 2 * std::max<uint32_t>(1, d->n_adjs)) cap <<= 1;
    std::vector<Adj> slots(cap);
    memset(slots.data(), 0, sizeof(Adj) * cap);
    uint32_t count = 0;
    for (uint32_t i = 0; i < d->n_adjs; i++) {
      const dp_adjacency_t &s = d->adjs[i];
      if (s.addr.family != 4 && s.addr.family != 6) return DP_EINVAL;
      uint8_t a[16] = {0};
      memcpy(a, s.addr.addr, s.addr.family == 6 ? 16 : 4);
      uint32_t w[4] = {be32(a), be32(a + 4), be32(a + 8), be32(a + 12)};
      uint32_t h = hmix(s.ifindex ^ ((uint32_t)s.addr.family << 24), w[0] ^ w[2], w[1] ^ w[3]) & (cap - 1);
      for (;;) {
        Adj &e = slots[h];
        if (!e.used) {
          e.used = 1; e.ifindex = s.ifindex; e.fam = s.addr.family;
          memcpy(e.addr, a, 16); memcpy(e.mac, s.mac, 6);
          count++;
          break;
        }
        if (e.ifindex == s.ifindex && e.fam == s.addr.family && memcmp(e.addr, a, 16) == 0) {
          memcpy(e.mac, s.mac, 6);  // HashMap insert replaces
          break;
        }
        h = (h + 1) & (cap - 1);
      }
    }
    im.adjs.slots = ib.put(slots);
    im.adjs.mask = cap - 1;
    im.adjs.count = count;
  }

  section("ifaces");
  // --- classifiers
  int rc;
  struct T { const dp_rule_t *r; uint32_t n; int fam; bool prio; int kind; Classifier *dst; };
  T tabs[6] = {
      {d->acl_v4, d->n_acl_v4, 4, false, 0, &im.acl[0]},
      {d->acl_v6, d->n_acl_v6, 6, false, 0, &im.acl[1]},
      {d->ff_remote_v4, d->n_ff_remote_v4, 4, true, 1, &im.ff_remote[0]},
      {d->ff_remote_v6, d->n_ff_remote_v6, 6, true, 1, &im.ff_remote[1]},
      {d->ff_local_v4, d->n_ff_local_v4, 4, true, 2, &im.ff_local[0]},
      {d->ff_local_v6, d->n_ff_local_v6, 6, true, 2, &im.ff_local[1]},
  };
  std::vector<KV> gkv[6];
  std::vector<std::vector<CRule>> keep(6);
  std::vector<const dp_rule_t *> ffr_order[2];
  std::vector<std::pair<uint64_t, const dp_rule_t *>> ffr_aux[2];
  for (int ti = 0; ti < 6; ti++)
    if ((rc = load_rules(tabs[ti].r, tabs[ti].n, tabs[ti].fam, tabs[ti].prio, tabs[ti].kind, keep[ti]))) return rc;
  // a flow-filter rule requiring port forwarding or masquerade (NatRequirement:
  // remote action2, local action)
  for (int ti = 2; ti < 6; ti++)
    for (uint32_t i = 0; i < tabs[ti].n; i++) {
      const uint32_t m = tabs[ti].kind == 1 ? tabs[ti].r[i].action2 : tabs[ti].r[i].action;
      if (m == DP_NAT_PORT_FORWARDING || m == DP_NAT_MASQUERADE) im.snat = 1;
      if (m == DP_NAT_MASQUERADE) im.masq = 1;
    }
  // the v6 window: the longest prefix (17..48 bits) holding every v6 rule
  // prefix of every classifier -- one site's rules share their top bits, and
  // the v6 address indexes then order the bits after them
  {
    int c = 48;
    bool any = false;
    u128 p0 = 0;
    for (int ti : {1, 3, 5})
      for (const CRule &cr : keep[ti])
        for (const dp_prefix_t *q : {&cr.r.src, &cr.r.dst}) {
          if (q->len == 0) continue;
          const u128 a = key128(6, q->addr);
          if (!any) p0 = a;
          any = true;
          const u128 x = a ^ p0;
          const int lcp = x == 0 ? 128 : ((uint64_t)(x >> 64) ? __builtin_clzll((uint64_t)(x >> 64))
                                                               : 64 + __builtin_clzll((uint64_t)x));
          c = std::min({c, (int)q->len, lcp});
        }
#ifdef DP_NO_V6_WINDOW
    any = false;
#endif
    g_v6w_c = any && c >= 17 ? c : 0;
    g_v6w_p = g_v6w_c ? p0 >> (128 - g_v6w_c) : 0;
    im.v6w_c = (uint32_t)g_v6w_c;
    im.v6w_p = (uint64_t)g_v6w_p;
  }
  for (int ti = 0; ti < 6; ti++) {
    auto &t = tabs[ti];
    bool ffr = ti == 2 || ti == 3;
    *t.dst = build_classifier(ib, keep[ti], t.fam, t.kind, &gkv[ti], ffr ? &ffr_order[ti - 2] : nullptr,
                              ffr ? &ffr_aux[ti - 2] : nullptr);
  }
  auto gkey = [](uint32_t a, uint32_t b, uint32_t c) {
    return ((unsigned __int128)a << 64) | ((unsigned __int128)b << 32) | c;
  };
  struct U128Hash { size_t operator()(unsigned __int128 x) const { return std::hash<uint64_t>()((uint64_t)x ^ (uint64_t)(x >> 64) * 0x9E3779B97F4A7C15ull); } };
  std::unordered_map<unsigned __int128, int32_t, U128Hash> gmap[6];
  for (int ti = 0; ti < 6; ti++)
    for (auto &e : gkv[ti]) gmap[ti][gkey(e.k0, e.k1, e.k2)] = (int32_t)e.v;
  auto group_of = [&](int ti, uint32_t a, uint32_t b) -> int32_t {
    auto it = gmap[ti].find(gkey(a, b, 0));
    return it == gmap[ti].end() ? -1 : it->second;
  };
  std::vector<KV> defkv;
  for (uint32_t i = 0; i < d->n_acl_defaults; i++)
    defkv.push_back(KV{d->acl_defaults[i].src_vni, d->acl_defaults[i].dst_vni, 0, d->acl_defaults[i].action + 1});
  im.acl_default = build_hash(ib, defkv);

  section("classifiers");
  // --- static NAT
  std::vector<NatTab> ntabs;
  std::vector<NatEnt> nents;
  std::vector<uint32_t> nprs;
  std::vector<NatRange> nranges;
  std::vector<KV> ntkv, pervni;
  // merge descriptors with the same key (PerVniTable semantics)
  std::vector<std::pair<KV, std::vector<const dp_nat_entry_t *>>> merged;
  std::unordered_map<std::string, size_t> midx;
  for (uint32_t i = 0; i < d->n_nat_tables; i++) {
    const dp_nat_table_t &t = d->nat_tables[i];
    if (t.kind > 1 || (uint64_t)t.first_entry + t.n_entries > d->n_nat_entries) return DP_EINVAL;
    KV k{t.kind, t.src_vni, t.kind ? t.dst_vni : 0, 0};
    std::string ks((const char *)&k, 12);
    auto it = midx.find(ks);
    if (it == midx.end()) { midx[ks] = merged.size(); merged.push_back({k, {}}); it = midx.find(ks); }
    for (uint32_t j = 0; j < t.n_entries; j++) merged[it->second].second.push_back(&d->nat_entries[t.first_entry + j]);
    pervni.push_back(KV{t.src_vni, 0, 0, 1});
  }
  for (auto &mt : merged) {
    // dedupe by prefix: last insert wins, position of first
    std::vector<const dp_nat_entry_t *> es;
    for (auto *e : mt.second) {
      if (e->prefix.family != 4 || !valid_prefix(e->prefix)) return DP_ENOTSUP;  // NAT44 only
      if ((uint64_t)e->first_port_range + e->n_port_ranges > d->n_nat_port_ranges) return DP_EINVAL;
      if ((uint64_t)e->first_range + e->n_ranges > d->n_nat_ranges) return DP_EINVAL;
      bool rep = false;
      for (auto &x : es)
        if (x->prefix.len == e->prefix.len && memcmp(x->prefix.addr, e->prefix.addr, 4) == 0) { x = e; rep = true; break; }
      if (!rep) es.push_back(e);
    }
    uint32_t base = (uint32_t)nents.size();
    for (auto *e : es) {
      NatEnt ne{};
      ne.net = be32(e->prefix.addr);
      ne.len = e->prefix.len;
      ne.is_pat = e->is_pat ? 1 : 0;
      ne.size_lo = (uint32_t)e->size;
      ne.size_hi = (uint32_t)(e->size >> 32);
      ne.first_pr = (uint32_t)nprs.size();
      ne.n_pr = e->n_port_ranges;
      uint64_t tot = 0;
      for (uint32_t k = 0; k < e->n_port_ranges; k++) {
        const dp_port_range_t &pr = d->nat_port_ranges[e->first_port_range + k];
        nprs.push_back((uint32_t)pr.lo | ((uint32_t)pr.hi << 16));
        tot += (uint64_t)pr.hi - pr.lo + 1;
      }
      ne.covers_all = (!e->is_pat || tot == 65536) ? 1 : 0;
      // one port range: kept in the entry itself (inl bit 1), no second read
      if (e->n_port_ranges == 1) {
        ne.first_pr = nprs.back();
        ne.inl |= 2;
      }
      std::vector<NatRange> rs;
      for (uint32_t k = 0; k < e->n_ranges; k++) {
        const dp_nat_range_t &s = d->nat_ranges[e->first_range + k];
        NatRange x{};
        x.olo_ip = be32(s.orig_lo_ip); x.ohi_ip = be32(s.orig_hi_ip);
        x.olo_port = s.orig_lo_port; x.ohi_port = s.orig_hi_port;
        x.tlo_ip = be32(s.tgt_lo_ip); x.thi_ip = be32(s.tgt_hi_ip);
        x.tlo_port = s.tgt_lo_port; x.thi_port = s.tgt_hi_port;
        x.offset = s.offset;
        rs.push_back(x);
      }
      std::stable_sort(rs.begin(), rs.end(), [](const NatRange &a, const NatRange &b) {
        if (a.olo_ip != b.olo_ip) return a.olo_ip < b.olo_ip;
        return a.olo_port < b.olo_port;
      });
      ne.first_range = (uint32_t)nranges.size();
      ne.n_ranges = (uint32_t)rs.size();
      if (rs.size() == 1 && rs[0].offset <= 0xffffffffull) {
        const NatRange &x = rs[0];
        ne.inl |= 1;
        ne.olo_ip = x.olo_ip; ne.ohi_ip = x.ohi_ip; ne.olo_port = x.olo_port; ne.ohi_port = x.ohi_port;
        ne.tlo_ip = x.tlo_ip; ne.thi_ip = x.thi_ip; ne.tlo_port = x.tlo_port; ne.thi_port = x.thi_port;
        ne.offset = (uint32_t)x.offset;
      }
      nranges.insert(nranges.end(), rs.begin(), rs.end());
      ne.parent = -1;
      nents.push_back(ne);
    }
    uint32_t cnt = (uint32_t)es.size();
    auto covers = [](const NatEnt &p, uint32_t a) {
      uint32_t m = p.len == 0 ? 0 : (0xffffffffu << (32 - p.len));
      return (a & m) == p.net;
    };
    for (uint32_t i = 0; i < cnt; i++) {
      NatEnt &e = nents[base + i];
      int best = -1;
      for (uint32_t j = 0; j < cnt; j++) {
        const NatEnt &f = nents[base + j];
        if (j == i || f.len >= e.len || !covers(f, e.net)) continue;
        if (best < 0 || f.len > nents[base + best].len) best = (int)j;
      }
      e.parent = best < 0 ? -1 : (int32_t)(base + best);
    }
    std::vector<uint64_t> bnd{0};
    for (uint32_t i = 0; i < cnt; i++) {
      const NatEnt &e = nents[base + i];
      bnd.push_back(e.net);
      uint64_t end = (uint64_t)e.net + (e.len == 0 ? (1ull << 32) : (1ull << (32 - e.len)));
      if (end <= 0xffffffffull) bnd.push_back(end);
    }
    std::sort(bnd.begin(), bnd.end());
    bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
    std::vector<uint32_t> b32;
    std::vector<int32_t> longest;
    for (uint64_t b : bnd) {
      b32.push_back((uint32_t)b);
      int best = -1;
      for (uint32_t i = 0; i < cnt; i++) {
        const NatEnt &e = nents[base + i];
        if (!covers(e, (uint32_t)b)) continue;
        if (best < 0 || e.len > nents[base + best].len) best = (int)i;
      }
      longest.push_back(best < 0 ? -1 : (int32_t)(base + best));
    }
    NatTab t{};
    t.n = (uint32_t)b32.size();
    if (t.n > 16) {
      // multibit table over the address intervals: leaf = longest entry + 1
      const int s0 = merged.size() > 128 ? 8 : 16;
      auto ivl = [&](uint64_t x) -> size_t {
        return (size_t)(std::upper_bound(b32.begin(), b32.end(), (uint32_t)x) - b32.begin()) - 1;
      };
      std::vector<uint32_t> blocks;
      std::function<uint32_t(uint64_t, int)> node = [&](uint64_t lo, int bits) -> uint32_t {
        size_t i0 = ivl(lo), i1 = ivl(lo + ((1ull << bits) - 1));
        if (i0 == i1) return DPD_LEAF | (uint32_t)(longest[i0] + 1);
        uint32_t ch[256];
        for (uint32_t c = 0; c < 256; c++) ch[c] = node(lo + ((uint64_t)c << (bits - 8)), bits - 8);
        uint32_t bi = (uint32_t)(blocks.size() / 256);
        blocks.insert(blocks.end(), ch, ch + 256);
        return bi;
      };
      std::vector<uint32_t> root((size_t)1 << s0);
      for (uint64_t b = 0; b < root.size(); b++) root[b] = node(b << (32 - s0), 32 - s0);
      if (blocks.empty()) blocks.push_back(0);
      t.root = ib.put(root);
      t.blocks = ib.put(blocks);
      t.s0 = (uint8_t)s0;
    } else {
      t.bounds = ib.put(b32);
      t.longest = ib.put(longest);
    }
    KV k = mt.first;
    k.v = (uint32_t)ntabs.size();
    ntkv.push_back(k);
    ntabs.push_back(t);
  }
  im.nat_tabs = build_hash(ib, ntkv);
  im.nat_pervni = build_hash(ib, pervni);

  section("nat");
  // --- per-VNI and per-VNI-pair contexts (precomputed joins)
  std::unordered_map<unsigned __int128, int32_t, U128Hash> ntmap;
  std::unordered_map<uint32_t, uint32_t> has_pervni;
  for (auto &e : ntkv) ntmap[gkey(e.k0, e.k1, e.k2)] = (int32_t)e.v;
  for (auto &e : pervni) has_pervni[e.k0] = 1;
  auto nat_tab = [&](uint32_t kind, uint32_t sv, uint32_t dv) -> int32_t {
    auto it = ntmap.find(gkey(kind, sv, dv));
    return it == ntmap.end() ? -1 : it->second;
  };
  // multibit index descriptors for the context records (Mbi)
  auto cls_mbi = [&](const Classifier &C, int32_t gi) {
    Mbi m{};
    if (gi < 0) return m;
    Group G;
    memcpy(&G, ib.b.data() + C.group_recs + (uint64_t)gi * sizeof(Group), sizeof(Group));
    if (G.mode != DPD_GROUP_LIST || !G.f[G.lfield].root) return m;
    const FieldIdx &F = G.f[G.lfield];
    m.root = (uint32_t)F.root; m.blocks = (uint32_t)F.blocks; m.s0 = F.s0; m.kbits = F.kbits;
    m.field = (uint8_t)G.lfield;
    return m;
  };
  // the second list index of a v4 ACL group (Group.lfield2)
  auto cls_mbi2 = [&](const Classifier &C, int32_t gi) {
    Mbi m{};
    if (gi < 0) return m;
    Group G;
    memcpy(&G, ib.b.data() + C.group_recs + (uint64_t)gi * sizeof(Group), sizeof(Group));
    if (G.mode != DPD_GROUP_LIST || !G.f[G.lfield].root || G.lfield2 == DPD_NO_FIELD || !G.f[G.lfield2].root)
      return m;
    const FieldIdx &F = G.f[G.lfield2];
    m.root = (uint32_t)F.root; m.blocks = (uint32_t)F.blocks; m.s0 = F.s0; m.kbits = F.kbits;
    m.field = (uint8_t)G.lfield2;
    return m;
  };
  auto nat_mbi = [&](int32_t ti) {
    Mbi m{};
    if (ti < 0 || !ntabs[ti].root || ntabs[ti].n == 0) return m;
    m.root = (uint32_t)ntabs[ti].root; m.blocks = (uint32_t)ntabs[ti].blocks; m.s0 = ntabs[ti].s0; m.kbits = 32;
    return m;
  };
  std::vector<VniRec> vrecs;
  std::vector<KV> vnikv2;
  for (uint32_t vni : vni_order) {
    VniRec r{};
    r.vni = vni;
    r.fib = vni2fib[vni];
    r.vrf_id = d->fibs[r.fib].vrf_id;
    r.ffr[0] = group_of(2, vni, 0);
    r.ffr[1] = group_of(3, vni, 0);
    r.nat_dst = nat_tab(0, vni, 0);
    r.pervni = has_pervni.count(vni) ? 1 : 0;
    r.ffr4 = cls_mbi(im.ff_remote[0], r.ffr[0]);
    r.ndst = nat_mbi(r.nat_dst);
    vnikv2.push_back(KV{vni, 0, 0, (uint32_t)vrecs.size()});
    vrecs.push_back(r);
  }
  {
    // the records are the slots of the VNI map (key vni, 0 = empty)
    uint32_t cap = 2;
    while (cap < 2 * std::max<size_t>(1, vrecs.size())) cap <<= 1;
    std::vector<VniRec> slots(cap);
    memset(slots.data(), 0, sizeof(VniRec) * cap);
    for (auto &r : vrecs) {
      if (r.vni == 0) return DP_EINVAL;
      uint32_t i = hmix(r.vni, 0, 0) & (cap - 1);
      while (slots[i].vni != 0) i = (i + 1) & (cap - 1);
      slots[i] = r;
    }
    im.vni_slots = ib.put(slots);
    im.vni_mask = cap - 1;
    im.n_vni_recs = (uint32_t)vrecs.size();
  }
  std::unordered_map<uint64_t, uint32_t> pidx;
  std::vector<PairRec> prs;
  std::vector<KV> pkv;
  std::unordered_map<uint64_t, uint32_t> defmap;
  for (auto &e : defkv) defmap[((uint64_t)e.k0 << 32) | e.k1] = e.v;
  auto pair_of = [&](uint32_t sv, uint32_t dv) -> uint32_t {
    uint64_t k = ((uint64_t)sv << 32) | dv;
    auto it = pidx.find(k);
    if (it != pidx.end()) return it->second;
    PairRec r{};
    r.ffl[0] = group_of(4, sv, dv);
    r.ffl[1] = group_of(5, sv, dv);
    r.acl[0] = group_of(0, sv, dv);
    r.acl[1] = group_of(1, sv, dv);
    auto dm = defmap.find(k);
    r.acl_def = dm == defmap.end() ? 0 : dm->second;
    r.nat_src = nat_tab(1, sv, dv);
    auto f = vni2fib.find(dv);
    r.dst_fib = f == vni2fib.end() ? -1 : (int32_t)f->second;
    r.dst_vni = dv;
    r.ffl4 = cls_mbi(im.ff_local[0], r.ffl[0]);
    r.acl4 = cls_mbi(im.acl[0], r.acl[0]);
    r.acl4b = cls_mbi2(im.acl[0], r.acl[0]);
    r.nsrc = nat_mbi(r.nat_src);
    if (r.dst_fib >= 0) { r.lpm4_direct = fibs[r.dst_fib].v4.direct; r.lpm4_dbits = fibs[r.dst_fib].v4.dbits;
                          r.lpm4_blocks = fibs[r.dst_fib].v4.blocks; }
    uint32_t id = (uint32_t)prs.size();
    pidx[k] = id;
    pkv.push_back(KV{sv, dv, 0, id});
    prs.push_back(r);
    return id;
  };
  for (int t = 0; t < 2; t++) {
    std::vector<uint32_t> aux;
    for (const dp_rule_t *r : ffr_order[t]) aux.push_back(pair_of(r->vni_a, r->action));
    im.ff_remote[t].aux = ib.put(aux);
    for (auto &pa : ffr_aux[t]) {
      uint32_t v = pair_of(pa.second->vni_a, pa.second->action);
      memcpy(ib.b.data() + pa.first, &v, 4);
    }
  }
  for (int ti : {0, 1, 4, 5})
    for (auto &e : gkv[ti]) if (e.k2 == 0) pair_of(e.k0, e.k1);
  for (auto &e : defkv) pair_of(e.k0, e.k1);
  for (auto &e : ntkv) if (e.k0 == 1) pair_of(e.k1, e.k2);
  im.pairs = build_hash(ib, pkv);
  im.pair_recs = ib.put(prs);
  im.n_pair_recs = (uint32_t)prs.size();
  {
    // the per-workgroup LDS copy of the context tables (dp_kernel.hip DP_CTX)
    auto a16 = [](uint64_t x) { return (x + 15) & ~15ull; };
    const uint64_t vni = a16((uint64_t)(im.vni_mask + 1) * sizeof(VniRec));
    const uint64_t psl = a16((uint64_t)(im.pairs.mask + 1) * sizeof(HashSlot));
    const uint64_t prc = a16((uint64_t)im.n_pair_recs * sizeof(PairRec));
    const uint64_t nh = a16((uint64_t)im.n_nh * sizeof(NhRec));
    // (only where packets read them: an image without VPC peerings routes
    // in the underlay, and there the copy cost C1 5 %)
    if (im.n_pair_recs && vni + psl + prc + nh <= DPD_CTX_MAX) {
      im.ctx_pslots = (uint32_t)vni;
      im.ctx_prec = (uint32_t)(vni + psl);
      im.ctx_nh = (uint32_t)(vni + psl + prc);
      im.ctx_bytes = (uint32_t)(vni + psl + prc + nh);
    }
  }
  im.nat_tab_recs = ib.put(ntabs);
  im.nat_ents = ib.put(nents);
  im.nat_prs = ib.put(nprs);
  im.nat_ranges = ib.put(nranges);

  section("contexts");
  // --- port forwarding (nat/src/portfw/portfwtable/)
  for (uint32_t i = 0; i < d->n_portfw; i++)
    if (!pf_rule_ok(d->portfw[i])) return DP_EINVAL;
  const PfLineage none;
  PfLineage L = pf_update(pf ? *pf : none, d->portfw, d->n_portfw);
  std::vector<PfEntry> ents = L.live;
  // lookup_cumulative (lpmmap.rs:108-116) over one key's entries: longest
  // prefix first, the first whose prefix holds the address and range the port
  std::stable_sort(ents.begin(), ents.end(), [](const PfEntry &a, const PfEntry &b) {
    if (a.r.src_vni != b.r.src_vni) return a.r.src_vni < b.r.src_vni;
    if (a.r.proto != b.r.proto) return a.r.proto < b.r.proto;
    return a.r.ext_prefix.len > b.r.ext_prefix.len;
  });
  std::vector<PfRuleRec> pfrecs;
  std::vector<KV> pkkv, pidkv;
  for (size_t i = 0; i < ents.size(); i++) {
    const dp_portfw_rule_t &r = ents[i].r;
    PfRuleRec q{};
    q.id = ents[i].id;
    q.src_vni = r.src_vni;
    q.dst_vni = r.dst_vni;
    q.proto = r.proto;
    q.fam = r.ext_prefix.family;
    q.plen = r.ext_prefix.len;
    q.ext_lo = r.ext_lo; q.ext_hi = r.ext_hi; q.int_lo = r.int_lo; q.int_hi = r.int_hi;
    be_words(r.ext_prefix, q.ext);
    be_words(r.int_prefix, q.inn);
    q.init_ns = (uint64_t)(r.init_timeout_s ? r.init_timeout_s : 10) * 1000000000ull;  // objects.rs:50-52
    q.estab_ns = (uint64_t)(r.estab_timeout_s ? r.estab_timeout_s : (r.proto == 6 ? 1800 : 30)) * 1000000000ull;
    if (i == 0 || ents[i - 1].r.src_vni != r.src_vni || ents[i - 1].r.proto != r.proto)
      pkkv.push_back(KV{r.src_vni, r.proto, 0, (uint32_t)i << 16});
    pkkv.back().v++;
    pidkv.push_back(KV{q.id, 0, 0, (uint32_t)i});
    pfrecs.push_back(q);
  }
  if (pfrecs.size() >= 65536) return DP_ENOTSUP;
  im.pf_keys = build_hash(ib, pkkv);
  im.pf_ids = build_hash(ib, pidkv);
  im.pf_rules = pfrecs.empty() ? ib.alloc(sizeof(PfRuleRec)) : ib.put(pfrecs);
  im.n_pf = (uint32_t)pfrecs.size();
  // do two rules' internal sides overlap (the same destination VPC, family
  // and protocol -- 0 any --, overlapping internal prefixes and port ranges)?
  // (within one rule the mapping is one to one)
  im.pf_overlap = 0;
  if (pfrecs.size() > 2048) {
    im.pf_overlap = 1;  // (not searched: assumed)
  } else {
    auto pre_meet = [](const PfRuleRec &a, const PfRuleRec &b) {
      const uint32_t len = std::min<uint32_t>(a.plen, b.plen);
      for (uint32_t w = 0; w < 4; w++) {
        const uint32_t lo = 32 * w;
        if (lo >= len) break;
        const uint32_t bits = std::min<uint32_t>(32, len - lo);
        const uint32_t m = bits == 32 ? 0xffffffffu : ~(0xffffffffu >> bits);
        if ((a.inn[w] ^ b.inn[w]) & m) return false;
      }
      return true;
    };
    for (size_t i = 0; i < pfrecs.size() && !im.pf_overlap; i++)
      for (size_t j = i + 1; j < pfrecs.size() && !im.pf_overlap; j++) {
        const PfRuleRec &a = pfrecs[i], &b = pfrecs[j];
        if (a.dst_vni != b.dst_vni || a.fam != b.fam) continue;
        if (a.proto && b.proto && a.proto != b.proto) continue;
        if (a.int_hi < b.int_lo || b.int_hi < a.int_lo) continue;
        if (pre_meet(a, b)) im.pf_overlap = 1;
      }
  }
  if (im.n_pf || d->n_masq) im.snat = 1;
  if (d->n_masq) im.masq = 1;

  section("portfw");
  // --- masquerade exposes (nat/src/masquerade/): validated and kept with the
  // image; each flow table builds its allocator from them (dp_masq.h)
  auto mc = std::make_shared<MasqConfig>();
  if (d->n_masq && (!d->masq || !d->masq_prefixes)) return DP_EINVAL;
  if (d->n_masq_claims && !d->masq_claims) return DP_EINVAL;
  auto put = [&](const void *x, size_t k) { mc->canon.append(static_cast<const char *>(x), k); };
  for (uint32_t i = 0; i < d->n_masq; i++) {
    const dp_masq_expose_t &x = d->masq[i];
    if (!x.src_vni || !x.dst_vni || x.src_vni == x.dst_vni || !x.n_public || !x.n_private) return DP_EINVAL;
    if ((uint64_t)x.first_prefix + x.n_private + x.n_public > d->n_masq_prefixes) return DP_EINVAL;
    if ((uint64_t)x.first_claim + x.n_claims > d->n_masq_claims) return DP_EINVAL;
    MasqExpose e;
    e.src_vni = x.src_vni;
    e.dst_vni = x.dst_vni;
    // the expose's idle timeout, by default 2 minutes (masquerade/state.rs)
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
    // canonical bytes: the same layout as the restatement's (a config is
    // "the same" when these match, absent a tag)
    put(&x.src_vni, 4); put(&x.dst_vni, 4); put(&e.idle_ns, 8);
    for (auto *v : {&e.priv, &e.pub}) {
      const uint32_t m = (uint32_t)v->size();
      put(&m, 4);
      for (auto &q : *v) put(&q, sizeof q);
    }
    const uint32_t m = (uint32_t)e.claims.size();
    put(&m, 4);
    for (auto &c : e.claims) put(&c, sizeof c);
    mc->exposes.push_back(std::move(e));
  }
  mc->tag = d->masq_config_tag;
  mc->randomize = d->masq_randomize != 0;
  mc->seed = d->masq_seed;
  ib.alloc(64);
  im.bytes = ib.b.size();
  // context records carry 32-bit image offsets (Mbi)
  if (im.bytes >= (1ull << 32)) return DP_ENOMEM;
  out.bytes.swap(ib.b);
  out.im = im;
  out.pt_nodes = pb.nodes.size();
  out.masq = mc;
  if (pf) *pf = std::move(L);
  return 0;
}

}  // namespace dpd

// Test introspection: classifier groups built in bit-vector ([0]) and
// candidate-list ([1]) form by the last image build on the calling thread.
// Test hook: classifier form for later image builds in this process (0 auto,
// 1 bit-vector, 2 candidate list).  Not part of the product ABI (dpgpu.h).
extern "C" void dpd_debug_set_classifier_form(int form) {
  dpd::g_cls_form.store(form >= 0 && form <= 2 ? form : 0, std::memory_order_relaxed);
}

extern "C" const char *dpd_debug_group_stats(void) { return dpd::g_group_stats.c_str(); }
extern "C" const char *dpd_debug_image_sections(void) { return dpd::g_sections.c_str(); }

extern "C" void dpd_debug_classifier_forms(uint32_t out[2]) {
  out[0] = dpd::g_forms[0];
  out[1] = dpd::g_forms[1];
}

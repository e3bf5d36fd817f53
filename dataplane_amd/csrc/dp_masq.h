// SPDX-License-Identifier: Apache-2.0
//
// Masquerade address / port allocator (nat/src/masquerade/apalloc/) as device
// state of a flow table.  One contiguous buffer holds the allocator's
// configuration (the PoolTable, its PoolSets, the disjoint PoolRegions with
// the port-forwarding claims on them) and its state (per region the address
// bitmap and the in-use list; per address in use its PortAllocator: 256 block
// flags, the current index, the thread block and, per allocated block, its
// usage bitmap).  The code below runs on the device (the burst's sequential
// NAT pass, the release of allocations whose flows leave the table) and on
// the host (a publish builds a replacement allocator and re-reserves the
// tuples of the flows it carries, masquerade/flows.rs:94-190), over the same
// layout.
//
// The reference's ownership (an AllocatedPort holds its block, a block its
// address: Arc back-references whose Drop frees the tuple, port_alloc.rs:
// 513-565, alloc.rs:322-326) becomes counts: live ports per block, live blocks
// per address.  A block whose last port goes is free again; an address whose
// last block goes returns to the bitmap and leaves the in-use list (the
// reference skips and later drops its Weak; the order of the others is the
// same).  Block i of an address covers ports [256 perm[i], 256 perm[i] + 255]:
// perm is the identity (randomize = false) or the permutation dpgpu.h defines
// from the allocator's seed and the address (randomize = true, drawn when the
// address is put to use, as PortAllocator::new shuffles, port_alloc.rs:
// 105-113).  One thread: ThreadPortMap is one slot per address.
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

namespace dpm {

constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kMagic = 0x4d415351u;  // "MASQ"

// AllocatorError (nat/src/masquerade/allocation.rs:12-36)
enum Err : uint32_t { OK = 0, NO_FREE_IP, NO_PORT_BLOCK, NO_FREE_PORT, PORT_ALLOC_FAILED,
                      PORT_RESERVATION_FAILED, INTERNAL, DENIED, NO_POOL_FOUND };
__host__ __device__ inline bool exhaustion(uint32_t e) {
  return e == NO_FREE_IP || e == NO_PORT_BLOCK || e == NO_FREE_PORT;
}

// Addresses are 128-bit numbers as 4 words, most significant first (v4: w[3]).
struct A128 {
  uint32_t w[4];
};
__host__ __device__ inline int a_cmp(const A128 &a, const A128 &b) {
  for (int i = 0; i < 4; i++)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
__host__ __device__ inline A128 a_add(const A128 &a, uint32_t o) {
  A128 r = a;
  uint64_t c = o;
  for (int i = 3; i >= 0 && c; i--) {
    const uint64_t v = (uint64_t)r.w[i] + c;
    r.w[i] = (uint32_t)v;
    c = v >> 32;
  }
  return r;
}
// b - a when it fits 32 bits (else kNone)
__host__ __device__ inline uint32_t a_off(const A128 &a, const A128 &b) {
  if (a_cmp(b, a) < 0) return kNone;
  uint64_t borrow = 0;
  uint32_t d[4];
  for (int i = 3; i >= 0; i--) {
    const uint64_t v = (uint64_t)b.w[i] - a.w[i] - borrow;
    d[i] = (uint32_t)v;
    borrow = (v >> 63) & 1;
  }
  return (d[0] | d[1] | d[2]) ? kNone : d[3];
}
// prefix of `len` bits of a `bits`-wide address (32 / 128) covers `x`
__host__ __device__ inline bool a_covers(const A128 &net, uint32_t len, uint32_t fam, const A128 &x) {
  const int base = fam == 4 ? 96 : 0;  // v4 lives in the low 32 bits
  for (int i = 0; i < 4; i++) {
    const int lo = 32 * i;
    const int bits = (int)len + base - lo;  // prefix bits within word i
    if (lo + 32 <= base) continue;
    const uint32_t m = bits >= 32 ? 0xffffffffu : bits <= 0 ? 0u : ~0u << (32 - bits);
    if ((net.w[i] ^ x.w[i]) & m) return false;
  }
  return true;
}

// PoolTable entry (apalloc/mod.rs:111-117, 142-202): a private range of one
// (protocol, source VPC, destination VPC) and the PoolSet serving it
struct Ent {
  A128 lo, hi;
  uint32_t set;
  uint32_t pad[3];
};
// (protocol | family << 8, src VPC, dst VPC) -> run of Ent (open addressing)
struct KeySlot {
  uint32_t proto, src, dst;  // dst bit 31: occupied
  uint32_t first, n, pad[3];
};
// PoolSet (alloc.rs:182-185): regions in try order, the expose's idle timeout
struct Set {
  uint64_t idle_ns;
  uint32_t first_reg, n_reg;  // into setreg[]
};
// PoolRegion + its NatPool (alloc.rs:336-345): configuration, then state
struct Region {
  uint32_t fam, cap, excl_wk, pad0;   // cap: offsets [0, cap) (DP_MASQ_REGION_ADDRS bound)
  A128 start, last;                   // the region's range
  uint32_t claim_first, claim_n;      // port-forwarding claims (ReservedPorts) of its owners
  uint32_t head, tail;                // in-use addresses, oldest first
  uint32_t bits;                      // first word of its free bitmap (1 = free offset)
  uint32_t hint;                      // no free bit below this word
  uint32_t pad1[2];
};
struct Claim {  // a (prefix, port range) of ReservedPorts (reserved.rs:23)
  A128 net;
  uint32_t fam, len;
  uint32_t lo, hi;
};
// An address in use: AllocatedIp + its PortAllocator (port_alloc.rs:84-93)
struct Addr {
  uint32_t region, offset, prev, next;
  uint32_t usable, live_blocks, nonfull;  // usable_blocks; alive blocks; alive blocks not full
  int32_t thread_block;                   // ThreadPortMap (-1: none)
  uint32_t cur;                           // current_alloc_index
  uint32_t pad[3];
  uint8_t bflag[256];                     // bit 0: free, bit 1: alive (an AllocatedPortBlock lives)
  uint8_t perm[256];                      // AllocatorPortBlock::random_index of block i
  uint8_t inv[256];                       // the block whose random_index is j
  uint16_t blive[256];                    // live ports of an alive block
  uint32_t bm[256][8];                    // Bitmap256 of an alive block
};

struct Header {
  uint32_t magic, gen;                    // gen: the allocator generation a flow's allocation names
  int64_t genid;                          // NatAllocator::genid
  uint32_t key_mask, n_keys;
  uint32_t n_regions, n_recs;
  uint32_t free_top, live;                // free-record stack top, addresses in use
  uint32_t max_live, randomize;           // MasqueradeConfig::randomize
  uint64_t o_keys, o_ents, o_sets, o_setreg, o_regions, o_claims, o_bits, o_free, o_recs;
  uint64_t bytes;
  uint64_t seed;                          // the permutations' seed (dpgpu.h masq_seed)
};

// A view of one allocator buffer (device or host memory).
struct View {
  uint8_t *b;
  __host__ __device__ Header &h() const { return *reinterpret_cast<Header *>(b); }
  __host__ __device__ KeySlot *keys() const { return reinterpret_cast<KeySlot *>(b + h().o_keys); }
  __host__ __device__ Ent *ents() const { return reinterpret_cast<Ent *>(b + h().o_ents); }
  __host__ __device__ Set *sets() const { return reinterpret_cast<Set *>(b + h().o_sets); }
  __host__ __device__ uint32_t *setreg() const { return reinterpret_cast<uint32_t *>(b + h().o_setreg); }
  __host__ __device__ Region *regions() const { return reinterpret_cast<Region *>(b + h().o_regions); }
  __host__ __device__ Claim *claims() const { return reinterpret_cast<Claim *>(b + h().o_claims); }
  __host__ __device__ uint32_t *bits() const { return reinterpret_cast<uint32_t *>(b + h().o_bits); }
  __host__ __device__ uint32_t *freestk() const { return reinterpret_cast<uint32_t *>(b + h().o_free); }
  __host__ __device__ Addr *recs() const { return reinterpret_cast<Addr *>(b + h().o_recs); }
};

__host__ __device__ inline uint32_t kmix(uint32_t a, uint32_t b, uint32_t c) {  // dpd::hmix
  uint32_t h = a * 0x9E3779B1u;
  h ^= (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

// PoolTable::get (apalloc/mod.rs:155-180): of the entries of this protocol and
// pair of VPCs covering the address, the one starting nearest to it, then the
// narrowest.  Returns the PoolSet, or kNone (Denied).
__host__ __device__ inline uint32_t lookup(const View &v, uint32_t proto, uint32_t src, uint32_t dst,
                                           const A128 &a) {
  const Header &H = v.h();
  if (!H.n_keys) return kNone;
  const KeySlot *ks = v.keys();
  uint32_t i = kmix(proto, src, dst) & H.key_mask;
  for (uint32_t p = 0; p <= H.key_mask; p++, i = (i + 1) & H.key_mask) {
    const KeySlot &k = ks[i];
    if (!(k.dst >> 31)) return kNone;
    if (k.proto != proto || k.src != src || (k.dst & 0x7fffffffu) != dst) continue;
    const Ent *e = v.ents() + k.first;
    uint32_t best = kNone;
    A128 bl{}, bh{};
    for (uint32_t j = 0; j < k.n; j++) {
      if (a_cmp(e[j].lo, a) > 0 || a_cmp(a, e[j].hi) > 0) continue;
      if (best == kNone || a_cmp(e[j].lo, bl) > 0 || (a_cmp(e[j].lo, bl) == 0 && a_cmp(e[j].hi, bh) < 0)) {
        best = e[j].set;
        bl = e[j].lo;
        bh = e[j].hi;
      }
    }
    return best;
  }
  return kNone;
}

__host__ __device__ inline A128 addr_of(const View &v, const Addr &r) {
  return a_add(v.regions()[r.region].start, r.offset);
}

// Bitmap256::for_block (port_alloc.rs:768-787): the region's claims covering
// the address, clipped to the block; port 0 when it may not be given out
__host__ __device__ inline void block_init(const View &v, const Region &R, const A128 &a, uint32_t base,
                                           bool reserve_null, uint32_t bm[8]) {
  for (int k = 0; k < 8; k++) bm[k] = 0;
  if (reserve_null && base == 0) bm[0] |= 1u;
  const Claim *C = v.claims() + R.claim_first;
  for (uint32_t c = 0; c < R.claim_n; c++) {
    if (C[c].fam != R.fam || !a_covers(C[c].net, C[c].len, C[c].fam, a)) continue;
    const uint32_t s = C[c].lo > base ? C[c].lo : base, e = C[c].hi < (base | 0xffu) ? C[c].hi : (base | 0xffu);
    for (uint32_t p = s; p <= e && s <= e; p++) bm[(p - base) >> 5] |= 1u << ((p - base) & 31);
  }
}
__host__ __device__ inline bool bm_full(const uint32_t bm[8]) {
  uint32_t x = 0xffffffffu;
  for (int k = 0; k < 8; k++) x &= bm[k];
  return x == 0xffffffffu;
}
// ReservedForAddr::contains (reserved.rs:95-99)
__host__ __device__ inline bool claimed(const View &v, const Region &R, const A128 &a, uint32_t port) {
  const Claim *C = v.claims() + R.claim_first;
  for (uint32_t c = 0; c < R.claim_n; c++)
    if (C[c].fam == R.fam && C[c].lo <= port && port <= C[c].hi && a_covers(C[c].net, C[c].len, C[c].fam, a))
      return true;
  return false;
}

__host__ __device__ inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// The order of an address's port blocks (dpgpu.h: the shuffle of
// PortAllocator::new, port_alloc.rs:105-113, drawn from the seed and the
// address); the identity without randomize
__host__ __device__ inline void block_order(const Header &H, const A128 &a, uint8_t perm[256], uint8_t inv[256]) {
  for (uint32_t i = 0; i < 256; i++) perm[i] = (uint8_t)i;
  if (H.randomize) {
    uint64_t x = H.seed;
    for (int k = 0; k < 4; k++) x = splitmix64(x ^ a.w[k]);
    for (uint32_t i = 255; i >= 1; i--) {
      x = splitmix64(x);
      const uint32_t j = (uint32_t)(x % (i + 1));
      const uint8_t t = perm[i];
      perm[i] = perm[j];
      perm[j] = t;
    }
  }
  for (uint32_t i = 0; i < 256; i++) inv[perm[i]] = (uint8_t)i;
}
// the first port of block i
__host__ __device__ inline uint32_t block_base(const Addr &A, uint32_t i) { return (uint32_t)A.perm[i] << 8; }

// NatPool::use_new_ip / reserve_from_pool's new address: an AllocatedIp with
// its PortAllocator::new (port_alloc.rs:100-145), at the back of in_use
__host__ __device__ inline uint32_t addr_new(const View &v, uint32_t region, uint32_t offset) {
  Header &H = v.h();
  if (!H.free_top || H.live >= H.max_live) return kNone;
  const uint32_t r = v.freestk()[--H.free_top];
  H.live++;
  Region &R = v.regions()[region];
  Addr &A = v.recs()[r];
  A.region = region;
  A.offset = offset;
  A.prev = R.tail;
  A.next = kNone;
  if (R.tail != kNone) v.recs()[R.tail].next = r;
  else R.head = r;
  R.tail = r;
  A.usable = 0;
  A.live_blocks = 0;
  A.nonfull = 0;
  A.thread_block = -1;
  A.cur = 0;
  const A128 a = a_add(R.start, offset);
  block_order(H, a, A.perm, A.inv);
  // what block_init reads for each of the 256 blocks, read once (the stores
  // below never change it; the compiler cannot know that): the region's
  // well-known exclusion and the ranges of the claims covering this address
  // (up to kC of them; more: block_init itself), the identity order without
  // randomize.  On the device each of those reads was a dependent round to
  // memory per block: ~300 us for one new address on the allocating lane.
  const bool excl = R.excl_wk, ident = !H.randomize;
  constexpr uint32_t kC = 8;
  uint32_t clo[kC], chi[kC], nc = 0;
  bool many = false;
  {
    const Claim *C = v.claims() + R.claim_first;
    const uint32_t n = R.claim_n, fam = R.fam;
    for (uint32_t c = 0; c < n; c++) {
      if (C[c].fam != fam || !a_covers(C[c].net, C[c].len, C[c].fam, a)) continue;
      if (nc == kC) { many = true; break; }
      clo[nc] = C[c].lo;
      chi[nc] = C[c].hi;
      nc++;
    }
  }
  uint32_t usable = 0;
  for (uint32_t i = 0; i < 256; i++) {
    const uint32_t base = ident ? i << 8 : block_base(A, i);
    bool off = excl && base < 1024;
    if (!off) {
      uint32_t bm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (many) {
        block_init(v, R, a, base, false, bm);
      } else {
        for (uint32_t c = 0; c < nc; c++) {
          const uint32_t s = clo[c] > base ? clo[c] : base, e = chi[c] < (base | 0xffu) ? chi[c] : (base | 0xffu);
          for (uint32_t p = s; p <= e && s <= e; p++) bm[(p - base) >> 5] |= 1u << ((p - base) & 31);
        }
      }
      off = bm_full(bm);
    }
    A.bflag[i] = off ? 0 : 1;
    A.blive[i] = 0;
    if (!off) usable++;
  }
  A.usable = usable;
  return r;
}
// Drop of the last AllocatedIp reference: the offset is free again
// (deallocate_from_pool, alloc.rs:422-433), the entry leaves in_use
__host__ __device__ inline void addr_kill(const View &v, uint32_t r) {
  Header &H = v.h();
  Addr &A = v.recs()[r];
  Region &R = v.regions()[A.region];
  if (A.prev != kNone) v.recs()[A.prev].next = A.next;
  else R.head = A.next;
  if (A.next != kNone) v.recs()[A.next].prev = A.prev;
  else R.tail = A.prev;
  uint32_t *bw = v.bits() + R.bits;
  bw[A.offset >> 5] |= 1u << (A.offset & 31);
  if ((A.offset >> 5) < R.hint) R.hint = A.offset >> 5;
  A.region = kNone;
  v.freestk()[H.free_top++] = r;
  H.live--;
}

// An AllocatedPortBlock comes to life (allocate_block /
// allocate_block_for_reservation, port_alloc.rs:238-262, 311-329)
__host__ __device__ inline void block_new(const View &v, uint32_t r, uint32_t idx, bool allow_null) {
  Addr &A = v.recs()[r];
  const Region &R = v.regions()[A.region];
  A.bflag[idx] = 2;  // alive, not free
  A.blive[idx] = 0;
  A.usable--;
  A.live_blocks++;
  block_init(v, R, a_add(R.start, A.offset), block_base(A, idx), !allow_null, A.bm[idx]);
  if (!bm_full(A.bm[idx])) A.nonfull++;
}
// The block's last port went (Drop of AllocatedPortBlock: deallocate_block,
// port_alloc.rs:200-212), and with its last block the address (unless
// `keep`: the caller kills it later -- releases run per address in parallel,
// the address list and bitmap are shared)
__host__ __device__ inline void block_die(const View &v, uint32_t r, uint32_t idx, bool keep = false) {
  Addr &A = v.recs()[r];
  if (!bm_full(A.bm[idx])) A.nonfull--;
  A.bflag[idx] = 1;  // free again
  A.usable++;
  if (--A.live_blocks == 0 && !keep) addr_kill(v, r);
}
// allocate_port_from_block (port_alloc.rs:449-471): the lowest free port
__host__ __device__ inline uint32_t block_take(const View &v, uint32_t r, uint32_t idx, bool allow_null,
                                               uint32_t &port) {
  Addr &A = v.recs()[r];
  uint32_t *bm = A.bm[idx];
  for (int k = 0; k < 8; k++) {
    if (bm[k] == 0xffffffffu) continue;
    const uint32_t off = 32 * k + (uint32_t)__builtin_ctz(~bm[k]);
    const uint32_t p = block_base(A, idx) + off;
    if (!allow_null && p == 0) return PORT_ALLOC_FAILED;  // new_port_checked (never: bit 0 is preset)
    bm[k] |= 1u << (off & 31);
    A.blive[idx]++;
    if (bm_full(bm)) A.nonfull--;
    port = p;
    return OK;
  }
  return NO_FREE_PORT;
}

// The releases of one block of one address, run beside other blocks'
// (dp_flows.hip fl_rel_run_k): the block's bitmap and live count are the
// caller's own, the address's counters are shared with the lanes of its other
// blocks (atomic).  Returns true when the address lost its last block (the
// caller kills it afterwards).
__device__ inline bool release_par(const View &v, uint32_t r, uint32_t port) {
  Addr &A = v.recs()[r];
  if (A.region == kNone) return false;
  const uint32_t idx = A.inv[port >> 8], off = port & 0xffu;
  if (!(A.bflag[idx] & 2)) return false;
  uint32_t *bm = A.bm[idx];
  if (!(bm[off >> 5] & (1u << (off & 31)))) return false;
  const bool was_full = bm_full(bm);
  bm[off >> 5] &= ~(1u << (off & 31));
  if (was_full) atomicAdd(&A.nonfull, 1u);
  if (--A.blive[idx] != 0) return false;
  // block_die, the address's counters shared
  atomicSub(&A.nonfull, 1u);  // (not full: a port just went)
  A.bflag[idx] = 1;
  atomicAdd(&A.usable, 1u);
  return atomicSub(&A.live_blocks, 1u) == 1u;
}

// Drop of an AllocatedPort (port_alloc.rs:553-565): the port, then possibly
// its block and address.  keep: as block_die; returns true when the address
// lost its last block (and was kept).
__host__ __device__ inline bool release(const View &v, uint32_t r, uint32_t port, bool keep = false) {
  if (r >= v.h().n_recs) return false;
  Addr &A = v.recs()[r];
  if (A.region == kNone) return false;
  const uint32_t idx = A.inv[port >> 8], off = port & 0xffu;
  if (!(A.bflag[idx] & 2)) return false;
  uint32_t *bm = A.bm[idx];
  if (!(bm[off >> 5] & (1u << (off & 31)))) return false;  // never taken (the reference logs it)
  const bool was_full = bm_full(bm);
  bm[off >> 5] &= ~(1u << (off & 31));
  if (was_full) A.nonfull++;
  if (--A.blive[idx] == 0) {
    block_die(v, r, idx, keep);
    return keep && A.live_blocks == 0;
  }
  return false;
}

// PortAllocator::allocate_port (port_alloc.rs:264-284): the thread block if it
// lives and is not full, else the next free block from current_alloc_index
__host__ __device__ inline uint32_t port_alloc(const View &v, uint32_t r, bool allow_null, uint32_t &port) {
  Addr &A = v.recs()[r];
  if (A.thread_block >= 0) {
    const uint32_t tb = (uint32_t)A.thread_block;
    if ((A.bflag[tb] & 2) && !bm_full(A.bm[tb])) return block_take(v, r, tb, allow_null, port);
  }
  uint32_t idx = kNone;
  for (uint32_t k = 0; k < 256; k++) {
    const uint32_t i = (A.cur + k) & 0xffu;
    if (A.bflag[i] & 1) { idx = i; break; }
  }
  if (idx == kNone) return NO_PORT_BLOCK;
  A.thread_block = (int32_t)idx;
  A.cur = idx;
  block_new(v, r, idx, allow_null);
  const uint32_t e = block_take(v, r, idx, allow_null, port);
  if (e != OK) block_die(v, r, idx);  // the new block drops at once
  return e;
}
__host__ __device__ inline bool has_free_ports(const Addr &A) { return A.usable > 0 || A.nonfull > 0; }

// IpAllocator::allocate (alloc.rs:113-127): the addresses in use in order,
// else the lowest free offset as a new address
__host__ __device__ inline uint32_t pool_alloc(const View &v, uint32_t region, bool allow_null, uint32_t &rec,
                                               uint32_t &port) {
  Region &R = v.regions()[region];
  uint32_t outcome = NO_FREE_IP;
  for (uint32_t r = R.head; r != kNone; r = v.recs()[r].next) {
    if (!has_free_ports(v.recs()[r])) continue;
    const uint32_t e = port_alloc(v, r, allow_null, port);
    if (e == OK) { rec = r; return OK; }
    if (e == NO_FREE_PORT) continue;
    outcome = e;
    break;
  }
  if (!exhaustion(outcome)) return outcome;
  uint32_t *bw = v.bits() + R.bits;
  const uint32_t words = (R.cap + 31) >> 5;
  uint32_t off = kNone;
  for (uint32_t w = R.hint; w < words; w++) {
    if (!bw[w]) continue;
    off = 32 * w + (uint32_t)__builtin_ctz(bw[w]);
    R.hint = w;
    break;
  }
  if (off == kNone) { R.hint = words; return NO_FREE_IP; }
  const uint32_t r = addr_new(v, region, off);
  if (r == kNone) return NO_FREE_IP;  // every address record in use (DP_MASQ_ADDRS)
  bw[off >> 5] &= ~(1u << (off & 31));
  const uint32_t e = port_alloc(v, r, allow_null, port);
  if (e != OK) {
    // the new address drops at once (a block that came and went took it along)
    if (v.recs()[r].region != kNone && v.recs()[r].live_blocks == 0) addr_kill(v, r);
    return e;
  }
  rec = r;
  return OK;
}
// PoolSet::allocate (alloc.rs:208-224)
__host__ __device__ inline uint32_t set_alloc(const View &v, uint32_t set, bool allow_null, uint32_t &rec,
                                              uint32_t &port) {
  const Set &S = v.sets()[set];
  uint32_t ex = OK;
  for (uint32_t j = 0; j < S.n_reg; j++) {
    const uint32_t e = pool_alloc(v, v.setreg()[S.first_reg + j], allow_null, rec, port);
    if (e == OK) return OK;
    if (exhaustion(e)) { ex = e; continue; }
    return e;
  }
  return ex == OK ? (uint32_t)NO_FREE_IP : ex;
}
// PoolSet::reserve -> IpAllocator::reserve -> PortAllocator::reserve_port
// (alloc.rs:140-147, 227-239, 437-478; port_alloc.rs:286-374)
__host__ __device__ inline uint32_t set_reserve(const View &v, uint32_t set, const A128 &a, uint32_t port, bool ident,
                                                uint32_t &rec) {
  const Set &S = v.sets()[set];
  uint32_t region = kNone;
  for (uint32_t j = 0; j < S.n_reg && region == kNone; j++) {
    const uint32_t g = v.setreg()[S.first_reg + j];
    const Region &R = v.regions()[g];
    if (a_cmp(R.start, a) <= 0 && a_cmp(a, R.last) <= 0) region = g;
  }
  if (region == kNone) return NO_POOL_FOUND;
  Region &R = v.regions()[region];
  const uint32_t off = a_off(R.start, a);
  if (off == kNone || off >= R.cap) return NO_POOL_FOUND;  // map_address: not an offset it serves
  uint32_t r = kNone;
  for (uint32_t x = R.head; x != kNone; x = v.recs()[x].next)
    if (v.recs()[x].offset == off) { r = x; break; }
  if (r == kNone) {
    r = addr_new(v, region, off);
    if (r == kNone) return NO_POOL_FOUND;
    v.bits()[R.bits + (off >> 5)] &= ~(1u << (off & 31));
  }
  Addr &A = v.recs()[r];
  uint32_t e = OK;
  const uint32_t idx = A.inv[port >> 8];  // try_to_reserve_block: the block covering the port
  if (R.excl_wk && port < 1024) e = DENIED;
  else if (claimed(v, R, a, port)) e = DENIED;
  else if (A.bflag[idx] & 1) {
    block_new(v, r, idx, ident);
  } else if (!(A.bflag[idx] & 2)) {
    e = PORT_RESERVATION_FAILED;  // neither free nor in the allocated map
  }
  if (e == OK) {
    uint32_t *bm = A.bm[idx];
    const uint32_t o = port & 0xffu;
    if (bm[o >> 5] & (1u << (o & 31))) {
      e = PORT_RESERVATION_FAILED;  // already handed out
      if (A.blive[idx] == 0) block_die(v, r, idx);
    } else {
      const bool full0 = bm_full(bm);
      bm[o >> 5] |= 1u << (o & 31);
      A.blive[idx]++;
      if (!full0 && bm_full(bm)) A.nonfull--;
    }
  }
  if (e != OK) {
    if (v.recs()[r].region != kNone && v.recs()[r].live_blocks == 0) addr_kill(v, r);
    return e;
  }
  rec = r;
  return OK;
}

}  // namespace dpm

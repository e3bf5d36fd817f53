// SPDX-License-Identifier: Apache-2.0
//
// MI355X (gfx950) per-burst packet pipeline kernel.
//
// One work-item per packet, 128-thread workgroups (2 wave64s).  Each
// work-item stages its frame's first WIN bytes into a private LDS slab with
// 16-byte global loads (the frame's header window; bytes beyond it are read
// from HBM directly), walks the stage sequence of the reference router
// pipeline (dataplane/src/packet_processor/mod.rs:130-145) against the
// device table image (dp_device.h), and serializes the result in place:
//  - patch mode (layout unchanged, the common case): only the changed fields
//    are stored (MACs, TTL, addresses, ports, checksums);
//  - rewrite mode (VXLAN encap, parse-limit quirks): the whole header stack
//    is re-emitted from the LDS snapshot as aligned dword stores.
// The L4 checksum is always fully recomputed over the payload, as
// Packet::serialize does (net/src/packet/mod.rs:342-354).
// DoneReason counts are reduced per workgroup in LDS, one atomic per bin.
#ifdef DP_EMU
#include DP_EMU  // tests/emu: host build of the same per-packet code (debug harness)
#else
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

#include "../../include/dpgpu.h"
#include "dp_device.h"
#include "dp_flow.h"
#include "dp_masq.h"

namespace {

using namespace dpd;

// Split build (Makefile): DP_PART k compiles pipeline instantiation k
// (1..6) or everything else (0); without DP_PART one unit holds all.
#ifndef DP_PART
#define DP_PART -1
#endif
#define DP_IN_PART(k) (DP_PART < 0 || DP_PART == (k))
// DP_V6W: the v6 window lookups (a v6 FIB's window table, the classifiers'
// v6 key window -- Image.v6w_fib / v6w_c) compiled in.  Parts 1 and 2 build
// the non-flow pipeline without them, parts 7 and 8 with them, and
// dpk_launch_pipeline picks by the image; every other unit has them.
#ifndef DP_V6W
#if DP_PART == 1 || DP_PART == 2 || DP_PART == 9 || DP_PART == 10 || DP_PART == 11 || DP_PART == 12
#define DP_V6W 0
#else
#define DP_V6W 1
#endif
#endif
// DP_SNAT: stateful NAT (port forwarding, masquerade: their records, the
// flow-filter and ICMP-error branches of flows with NAT state) compiled into
// the flows variant.  Parts 9 and 10 build the flows first pass without it
// (and without the v6 window lookups) for images that configure no stateful
// NAT served by flow tables that never held NAT state (dpk_launch_pipeline_flows).
#ifndef DP_SNAT
#if DP_PART == 9 || DP_PART == 10
#define DP_SNAT 0
#else
#define DP_SNAT 1
#endif
#endif
constexpr bool SNAT = DP_SNAT;
// DP_CTX: the context tables (VNI slots, pair map, PairRecs, NhRecs) read
// from a per-workgroup LDS copy (Image.ctx_bytes > 0).  Parts 1, 2 (and 7,
// 8 with the v6 windows) build the non-flow pipeline so, at 256 work-items
// per workgroup (the copy is amortised over more packets and three
// workgroups' LDS still fit a CU at 3 waves per SIMD); parts 11, 12 (13, 14)
// without it, for images whose context tables do not fit DPD_CTX_MAX.  The
// lean flows units (9, 10) have it too: an image whose tables do not fit
// runs the full flows variant.
#ifndef DP_CTX
#if DP_PART == 1 || DP_PART == 2 || DP_PART == 7 || DP_PART == 8 || DP_PART == 9 || DP_PART == 10 || \
    DP_PART == 15 || DP_PART == 16
#define DP_CTX 1
#else
#define DP_CTX 0
#endif
#endif
#ifndef DP_TPB
#if DP_CTX
#define DP_TPB 256
#else
#define DP_TPB 128
#endif
#endif
constexpr int TPB = DP_TPB;  // work-items (packets) per workgroup
// LDS pointers carry their address space explicitly so every access is a
// ds_read/ds_write (a generic pointer would turn them into flat loads)
#ifdef DP_EMU
#define LDS_AS
#else
#define LDS_AS __attribute__((address_space(3)))
#endif
typedef LDS_AS uint8_t lds_u8;
typedef LDS_AS uint32_t lds_u32;
// Dependent-load round trips per packet and stage (host emulation only,
// -DDP_TRIPS; scripts/trips.py): the chain-length model of the kernel.
#if defined(DP_EMU) && defined(DP_TRIPS)
thread_local uint16_t dp_trip[8];
thread_local int dp_trip_st;
#define TRIP_ST(x) (dp_trip_st = (x))
#define TRIP() (dp_trip[dp_trip_st]++)
#else
#define TRIP_ST(x) ((void)0)
#define TRIP() ((void)0)
#endif
// Wave-level loop iterations on the GPU (diagnostic build -DDP_TIMING -DDP_GPU_TRIPS):
// the first active lane of the wave counts one iteration into g_stage_cycles[k]
#if defined(DP_TIMING) && defined(DP_GPU_TRIPS) && !defined(DP_EMU)
#define GTRIP(k) do { if ((int)threadIdx.x % 64 == __ffsll((long long)__ballot(1)) - 1) atomicAdd(&g_stage_cycles[k], 1ull); } while (0)
#else
#define GTRIP(k) ((void)0)
#endif
// Optional per-stage wave timing (build with -DDP_TIMING; scripts/stage_timing.py)
#if defined(DP_TIMING) && !defined(DP_EMU)
__device__ unsigned long long g_stage_cycles[16];
#define TS_DECL uint64_t ts_acc[12] = {0}; uint64_t ts_last = clock64();
#define TS(k) do { uint64_t ts_now = clock64(); ts_acc[k] += ts_now - ts_last; ts_last = ts_now; } while (0)
#define TS_FLUSH() do { if ((threadIdx.x & 63) == 0) for (int q = 0; q < 12; q++) atomicAdd(&g_stage_cycles[q], (unsigned long long)ts_acc[q]); } while (0)
#else
#define TS_DECL
#define TS(k) do {} while (0)
#define TS_FLUSH() do {} while (0)
#endif
// LDS per work-item: the header window slab + the hash-input scratch.
// 160 B per work-item (WIN 96 + 4 + 60) lets 8 blocks of 128 share a CU's
// 160 KiB: 4 waves per SIMD, matching the 128-VGPR budget of DP_WAVES 4.
#ifndef DP_WIN
#define DP_WIN 96
#endif
#ifndef DP_HS
#define DP_HS 76
#endif
#ifndef DP_CAND4
#define DP_CAND4 2  // v4 classifier candidates fetched per round trip (2 or 4; 4 measured slower)
#endif
#ifndef DP_WAVES
#define DP_WAVES 3
#endif
// DP_PERSIST: the non-flow pipeline kernel's workgroups stay resident and take
// chunk after chunk (pipeline_grid); A/B flag
#ifndef DP_PERSIST
#define DP_PERSIST 0
#endif
constexpr int WIN = DP_WIN;       // header window bytes per packet (rest read from HBM)
constexpr int SLAB = WIN + 4;     // odd dword stride: conflict-free byte reads
constexpr int HS = DP_HS;         // hash input scratch (packet_hash_vxlan's stream <= 75 B)
constexpr uint8_t DONE_NONE = 255;
// out-of-line cold paths (the emulator inlines freely, except its
// DP_EMU_OUTLINE build, which keeps every function out of line so the CPU
// suite runs the call shape of the device code: tests/emu libdpemu_outline.so)
#if defined(DP_EMU) && !defined(DP_EMU_OUTLINE)
#define DP_COLD
#else
#define DP_COLD __attribute__((noinline))
#endif
// the bit-vector classifier (classify_bv): out of line unless DP_BV_INLINE
#if defined(DP_BV_INLINE) && !defined(DP_EMU_OUTLINE)
#define DP_BV __forceinline__
#else
#define DP_BV DP_COLD
#endif

// ---------------------------------------------------------------------------
// Wave-aggregated counters
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// The next index of a burst-wide counter for each active lane that wants one
// (want): one atomic per wave, not one per lane -- lanes of a whole chip
// adding to one word are served one by one at its L2 channel.  Every active
// lane calls it; a lane that does not want one gets an unspecified value.
__device__ __forceinline__ uint32_t wave_claim(uint32_t *ctr, bool want) {
#ifdef DP_EMU  // one lane at a time
  return want ? atomicAdd(ctr, 1u) : 0u;
#else
  const uint64_t m = __ballot(want);
  if (!m) return 0;
  const int lane = threadIdx.x & 63, leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  return (uint32_t)__shfl((int)base, leader) + (uint32_t)__popcll(m & lanes_below(lane));
#endif
}

// ---------------------------------------------------------------------------
// Image access
// ---------------------------------------------------------------------------
struct ImgBase {
  const uint8_t *base;
  template <class T> __device__ __forceinline__ const T *at(uint64_t off) const {
    return reinterpret_cast<const T *>(base + off);
  }
};
struct Img : ImgBase {
  const Image &im;  // in HBM on the device (read where used), host memory in the emulator
  const LDS_AS uint8_t *ctx = nullptr;  // DP_CTX: the workgroup's copy of the context tables
  __device__ __forceinline__ Img(const uint8_t *b, const Image &i) : ImgBase{b}, im(i) {}
  __device__ __forceinline__ Img(const uint8_t *b, const Image &i, const LDS_AS uint8_t *c)
      : ImgBase{b}, im(i), ctx(c) {}
};
// The context tables, from the workgroup's LDS copy (DP_CTX) or HBM
#if DP_CTX
#define CTX_AS LDS_AS
#define CTX_TAB(T, lds_off, hbm_off) reinterpret_cast<const CTX_AS T *>(g.ctx + (lds_off))
#else
#define CTX_AS
#define CTX_TAB(T, lds_off, hbm_off) g.at<T>(hbm_off)
#endif
// a record of a context table as a value (DP_CTX: word by word out of LDS;
// the compiler drops the words nobody reads), else a reference into HBM
#if DP_CTX
template <class T> __device__ __forceinline__ T ctx_val(const CTX_AS T &x) {
  static_assert(sizeof(T) % 4 == 0, "word copy");
  T r;
  const CTX_AS uint32_t *src = reinterpret_cast<const CTX_AS uint32_t *>(&x);
  uint32_t *dst = reinterpret_cast<uint32_t *>(&r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / 4); k++) dst[k] = src[k];
  return r;
}
#define CTX_REC(T, lds_off, hbm_off, idx) ctx_val(CTX_TAB(T, lds_off, hbm_off)[idx])
#else
#define CTX_REC(T, lds_off, hbm_off, idx) g.at<T>(hbm_off)[idx]
#endif
#define VNI_REC(idx) CTX_REC(VniRec, 0, g.im.vni_slots, idx)
#define PAIR_REC(idx) CTX_REC(PairRec, g.im.ctx_prec, g.im.pair_recs, idx)

template <class SP>
__device__ __forceinline__ bool hash_probe(SP s, uint32_t mask, uint32_t k0, uint32_t k1, uint32_t k2,
                                           uint32_t &val) {
  uint32_t key2 = k2 | 0x80000000u;
  uint32_t i = hmix(k0, k1, k2) & mask;
  for (uint32_t probe = 0; probe <= mask; probe++) {
    TRIP();
    const uint32_t e2 = s[i].k2;
    if (!(e2 & 0x80000000u)) return false;
    if (s[i].k0 == k0 && s[i].k1 == k1 && e2 == key2) { val = s[i].val; return true; }
    i = (i + 1) & mask;
  }
  return false;
}
__device__ __forceinline__ bool hash_find(const Img &g, const HashMap &m, uint32_t k0,
                                          uint32_t k1, uint32_t k2, uint32_t &val) {
  if (m.count == 0) return false;
  return hash_probe(g.at<HashSlot>(m.slots), m.mask, k0, k1, k2, val);
}
// the (src VNI, dst VNI) -> PairRec map (a context table)
__device__ __forceinline__ bool pair_find(const Img &g, uint32_t k0, uint32_t k1, uint32_t &val) {
  if (g.im.pairs.count == 0) return false;
  return hash_probe(CTX_TAB(HashSlot, g.im.ctx_pslots, g.im.pairs.slots), g.im.pairs.mask, k0, k1, 0, val);
}

// ---------------------------------------------------------------------------
// Frame window: byte f of the frame is slab[shift + f] if inside the window,
// else read from HBM.
// ---------------------------------------------------------------------------
struct Frame {
  lds_u8 *lds;      // this work-item's slab
  lds_u8 *hs;       // this work-item's 64-byte LDS hash scratch
  uint8_t *g;       // frame start in HBM
  int shift;        // frame start & 15
  int len;
  // The whole frame is inside the window (shift + len <= WIN) at an even
  // window position: every read is an LDS read, and the 16-bit fields (all at
  // even frame offsets) are single 16-bit LDS accesses.  process_packet is inlined twice, with this a compile-time
  // true and false; a wave whose frames all fit runs the first copy, which
  // has none of the per-byte window tests and HBM fallbacks.
  bool inwin;
  // The LDS read is unconditional (clamped index) so the compiler keeps it a
  // ds_read and never fuses the two loads into one generic (flat) load
  // through a select of pointers; the HBM read stays behind a branch.
  __device__ __forceinline__ uint8_t b(int f) const {
    int o = shift + f;
#ifdef DP_EMU
    if (inwin && (o < 0 || o >= WIN)) __builtin_trap();
#endif
    if (inwin) return lds[o];
    uint8_t v = lds[o < WIN ? o : 0];
    if (o >= WIN) v = g[f];
    return v;
  }
  __device__ __forceinline__ uint16_t be16(int f) const {
#ifdef DP_EMU
    if (inwin && (f & 1)) __builtin_trap();
#endif
    if (inwin) {
      const uint32_t x = *reinterpret_cast<const LDS_AS uint16_t *>(lds + shift + f);
      return (uint16_t)((x << 8) | (x >> 8));
    }
    return (uint16_t)((b(f) << 8) | b(f + 1));
  }
  __device__ __forceinline__ uint32_t be32(int f) const {
    if (inwin) return ((uint32_t)be16(f) << 16) | be16(f + 2);
    return ((uint32_t)b(f) << 24) | ((uint32_t)b(f + 1) << 16) | ((uint32_t)b(f + 2) << 8) | b(f + 3);
  }
};

__device__ __forceinline__ uint64_t mac_at(const Frame &F, int f) {
  uint64_t m = 0;
  for (int i = 0; i < 6; i++) m = (m << 8) | F.b(f + i);
  return m;
}
__device__ __forceinline__ uint64_t load_mac(const uint8_t *p) {
  uint64_t m = 0;
  for (int i = 0; i < 6; i++) m = (m << 8) | p[i];
  return m;
}
__device__ __forceinline__ uint8_t mac_b(uint64_t m, int i) { return (uint8_t)(m >> (40 - 8 * i)); }

// Frame byte f lives at window position shift + f when 0 <= shift + f < WIN
// (the LDS copy, written back by flush_window); any other byte is written
// straight to the burst buffer.  Reads (F.b) see both.
// wput8_any: any byte of the slot (an encap prepend may start before the
// frame); wput8: a byte of the frame itself (0 <= f < len), an LDS store
// with no test when the whole frame is in the window.
__device__ __forceinline__ void wput8_any(const Frame &F, int f, uint32_t v) {
  const int o = F.shift + f;
  if ((unsigned)o < (unsigned)WIN) F.lds[o] = (uint8_t)v;
  else F.g[f] = (uint8_t)v;
}
__device__ __forceinline__ void wput8(const Frame &F, int f, uint32_t v) {
#ifdef DP_EMU
  if (F.inwin && (f < 0 || f >= F.len)) __builtin_trap();
#endif
  if (F.inwin) F.lds[F.shift + f] = (uint8_t)v;
  else wput8_any(F, f, v);
}
__device__ __forceinline__ void wput16(const Frame &F, int f, uint32_t v) {
  if (F.inwin) {
#ifdef DP_EMU
    if (f < 0 || f + 2 > F.len || (f & 1)) __builtin_trap();
#endif
    *reinterpret_cast<LDS_AS uint16_t *>(F.lds + F.shift + f) = (uint16_t)(((v & 0xff) << 8) | ((v >> 8) & 0xff));
    return;
  }
  wput8(F, f, v >> 8); wput8(F, f + 1, v);
}
__device__ __forceinline__ void wput32(const Frame &F, int f, uint32_t v) { wput16(F, f, v >> 16); wput16(F, f + 2, v); }

// ---------------------------------------------------------------------------
// Parsed header stack (offsets are frame-relative)
// ---------------------------------------------------------------------------
enum { L4_NONE = 0, L4_TCP = 1, L4_UDP = 2, L4_ICMP4 = 3, L4_ICMP6 = 4 };
enum { HK_NONE = 0, HK_VLAN, HK_V4, HK_V6, HK_EXT_RAW, HK_EXT_FRAG, HK_EXT_AUTH, HK_TCP, HK_UDP,
       HK_ICMP4, HK_ICMP6, HK_VXLAN };

struct Hdr {
  int hb;           // header stack start (eth)
  int nvlan;
  int net;          // 0 / 4 / 6
  int net_off, net_hlen;
  int next;         // number of kept ext headers
  int ext_off[3];
  uint8_t ext_kind[3];
  int ext_len;      // bytes of kept ext headers
  int l4, l4_off, l4_hlen;
  bool vx;
  int vx_off;
  uint32_t vni;
  int consumed;     // bytes consumed from hb
  int size;         // deparse size of the kept stack
  uint32_t emb;     // ICMP error message's embedded headers (emb_pack), 0: none
};

// try to parse one header of kind `k` at frame offset `pos`; returns its
// length (0 on failure)
__device__ __forceinline__ int try_parse(const Frame &F, int k, int pos, uint32_t &aux) {
  int rem = F.len - pos;
  switch (k) {
    case HK_VLAN: {  // Vlan::parse: VID 0 / 4095 invalid
      if (rem < 4) return 0;
      uint16_t vid = F.be16(pos) & 0x0fff;
      if (vid == 0 || vid == 4095) return 0;
      return 4;
    }
    case HK_V4: {  // Ipv4HeaderSlice::from_slice + unicast source
      if (rem < 20) return 0;
      uint8_t v = F.b(pos);
      if ((v >> 4) != 4) return 0;
      int ihl = v & 0xf;
      if (ihl < 5) return 0;
      int hl = ihl * 4;
      if (rem < hl) return 0;
      if (F.be16(pos + 2) < hl) return 0;
      uint32_t src = F.be32(pos + 12);
      if ((src >> 28) == 0xe || src == 0xffffffffu) return 0;
      return hl;
    }
    case HK_V6: {
      if (rem < 40) return 0;
      if ((F.b(pos) >> 4) != 6) return 0;
      if (F.b(pos + 8) == 0xff) return 0;
      return 40;
    }
    case HK_EXT_RAW: {
      if (rem < 8) return 0;
      int n = ((int)F.b(pos + 1) + 1) * 8;
      return rem < n ? 0 : n;
    }
    case HK_EXT_FRAG: return rem < 8 ? 0 : 8;
    case HK_EXT_AUTH: {
      if (rem < 12) return 0;
      uint8_t pl = F.b(pos + 1);
      if (pl == 0) return 0;
      int n = ((int)pl + 2) * 4;
      return rem < n ? 0 : n;
    }
    case HK_TCP: {
      if (rem < 20) return 0;
      int doff = F.b(pos + 12) >> 4;
      if (doff < 5 || rem < doff * 4) return 0;
      if (F.be16(pos) == 0 || F.be16(pos + 2) == 0) return 0;
      return doff * 4;
    }
    case HK_UDP: {
      if (rem < 8) return 0;
      if (F.be16(pos) == 0 || F.be16(pos + 2) == 0) return 0;
      return 8;
    }
    case HK_ICMP4: {
      if (rem < 8) return 0;
      uint8_t t = F.b(pos), c = F.b(pos + 1);
      int n = ((t == 13 || t == 14) && c == 0) ? 20 : 8;
      return rem < n ? 0 : n;
    }
    case HK_ICMP6: return rem < 8 ? 0 : 8;
    case HK_VXLAN: {
      if (rem < 8) return 0;
      if ((F.b(pos) & 0x08) != 0x08) return 0;
      if (F.b(pos + 1) | F.b(pos + 2) | F.b(pos + 3) | F.b(pos + 7)) return 0;
      uint32_t v = ((uint32_t)F.b(pos + 4) << 16) | ((uint32_t)F.b(pos + 5) << 8) | F.b(pos + 6);
      if (v == 0) return 0;
      aux = v;
      return 8;
    }
  }
  return 0;
}

__device__ __forceinline__ int kind_of_ethertype(uint16_t et) {
  if (et == 0x0800) return HK_V4;
  if (et == 0x86dd) return HK_V6;
  if (et == 0x8100 || et == 0x9100 || et == 0x88a8) return HK_VLAN;
  return HK_NONE;
}

// next header kind after an IP-ish header given proto, v4 / v6 context
__device__ __forceinline__ int kind_of_proto(uint8_t p, bool v6) {
  switch (p) {
    case 6: return HK_TCP;
    case 17: return HK_UDP;
    case 1: return v6 ? HK_NONE : HK_ICMP4;
    case 58: return v6 ? HK_ICMP6 : HK_NONE;
    case 51: return HK_EXT_AUTH;
    case 0: case 43: case 60: return v6 ? HK_EXT_RAW : HK_NONE;
    case 44: return v6 ? HK_EXT_FRAG : HK_NONE;
  }
  return HK_NONE;
}

// ---------------------------------------------------------------------------
// ICMP error messages (cold paths: only such packets reach them)
// ---------------------------------------------------------------------------
// Error message types as the reference sees them: etherparse's decoded
// type/code pairs mapped through net/src/icmp4/mod.rs:406-465 and
// net/src/icmp6/mod.rs:396-459 (a Redirect with a non-unicast gateway and a
// Packet Too Big below MTU 1280 are Unknown), error classes
// icmp4/mod.rs:555-563, icmp6/mod.rs:577-585.
__device__ __forceinline__ bool icmp_err_at(const Frame &F, int o, bool v6) {
  const uint8_t t = F.b(o), c = F.b(o + 1);
  if (!v6) {
    if (t == 3) return c <= 15;
    if (t == 5) {
      if (c > 3) return false;
      const uint32_t gw = F.be32(o + 4);
      return !((gw >> 28) == 0xe || gw == 0xffffffffu);
    }
    if (t == 11) return c <= 1;
    if (t == 12) return c <= 2;
    return false;
  }
  if (t == 1) return c <= 6;
  if (t == 2) return c == 0 && F.be32(o + 4) >= 1280;
  if (t == 3) return c <= 1;
  if (t == 4) return c <= 10;
  return false;
}

// Embedded headers of an ICMP error message (EmbeddedHeaders,
// net/src/headers/embedded.rs:43-48): frame offsets of the IP header, the
// kept extension headers and the (possibly truncated) transport header.
struct Emb {
  int off, net, net_hlen;
  int next, ext_len;
  int ext_off[3];
  uint8_t ext_kind[3];
  int tk;            // L4_* (L4_NONE: none)
  bool full;         // a full transport header (else a partial one: every remaining byte)
  int t_off, t_len;
  int consumed, rec;  // bytes consumed / written back by the deparse
};

// TruncatedTcp / TruncatedUdp / TruncatedIcmp4 / TruncatedIcmp6::parse
// (tcp/truncated.rs:193-214, udp/truncated.rs, icmp4/truncated.rs:200-221):
// the full header, else -- on a length shortfall only -- a partial header of
// every remaining byte (TCP/UDP: >= 4 bytes and non-zero ports; ICMP: >= 2).
// Returns the length (0: no transport), `full` tells which.
__device__ __forceinline__ int trunc_transport(const Frame &F, int pos, int k, bool &full) {
  const int rem = F.len - pos;
  uint32_t aux = 0;
  full = false;
  if (k == HK_TCP) {
    bool short_ = rem < 20;
    if (!short_) {
      const int doff = F.b(pos + 12) >> 4;
      if (doff < 5) return 0;
      short_ = rem < doff * 4;
    }
    if (!short_) { full = true; return try_parse(F, HK_TCP, pos, aux); }
  } else if (k == HK_UDP) {
    if (rem >= 8) { full = true; return try_parse(F, HK_UDP, pos, aux); }
  } else {
    const int n = try_parse(F, k, pos, aux);
    if (n) { full = true; return n; }
    return rem >= 2 ? rem : 0;
  }
  if (rem < 4 || F.be16(pos) == 0 || F.be16(pos + 2) == 0) return 0;
  return rem;
}

// EmbeddedHeaders::parse_with (embedded.rs:289-397) at `pos`: the IP header
// (else no embedded headers: false), then the embedded-payload dispatch of
// ipv4/mod.rs:320-331, ipv6/mod.rs:266-287, ipv6/ext_parse.rs:46-69,
// ip_auth/v4.rs:67-87, with the main loop's parse-then-record order (an
// extension header past MAX_NET_EXTENSIONS ends the loop after its successor
// was consumed).
__device__ __forceinline__ bool emb_parse(const Frame &F, int pos, bool v6, Emb &E) {
  uint32_t aux = 0;
  E.off = pos; E.net = v6 ? 6 : 4; E.next = 0; E.ext_len = 0; E.tk = L4_NONE; E.full = false;
  E.t_off = E.t_len = 0;
  E.net_hlen = try_parse(F, v6 ? HK_V6 : HK_V4, pos, aux);
  if (!E.net_hlen) return false;
  uint8_t nh = v6 ? F.b(pos + 6) : F.b(pos + 9);
  int p = pos + E.net_hlen;
  int prior = 0;  // 0 IP, 1 extension header, 2 transport
  int prior_off = 0, prior_len = 0, prior_kind = 0;
  bool prior_full = false;
  for (int guard = 0; guard < 8; guard++) {
    int next = -1, nlen = 0, nkind = 0, noff = p;
    bool nfull = false;
    if (prior != 2) {
      int k = HK_NONE;
      switch (nh) {
        case 6: k = HK_TCP; break;
        case 17: k = HK_UDP; break;
        case 1: k = v6 ? HK_NONE : HK_ICMP4; break;
        case 58: k = v6 ? HK_ICMP6 : HK_NONE; break;
        case 51: k = HK_EXT_AUTH; break;
        case 0: case 43: case 60: k = v6 ? HK_EXT_RAW : HK_NONE; break;
        case 44: k = v6 ? HK_EXT_FRAG : HK_NONE; break;
      }
      if (k == HK_TCP || k == HK_UDP || k == HK_ICMP4 || k == HK_ICMP6) {
        nlen = trunc_transport(F, p, k, nfull);
        next = nlen ? 2 : -1;
      } else if (k != HK_NONE) {
        nlen = try_parse(F, k, p, aux);
        next = nlen ? 1 : -1;
      }
      nkind = k;
      if (next >= 0) p += nlen;
    }
    bool brk = false;
    if (prior == 1) {
      if (E.next < 3) {
        E.ext_off[E.next] = prior_off; E.ext_kind[E.next] = (uint8_t)prior_kind;
        E.ext_len += prior_len;
        E.next++;
      } else {
        brk = true;
      }
    } else if (prior == 2) {
      E.tk = prior_kind == HK_TCP ? L4_TCP : prior_kind == HK_UDP ? L4_UDP
                                                                   : prior_kind == HK_ICMP4 ? L4_ICMP4 : L4_ICMP6;
      E.full = prior_full; E.t_off = prior_off; E.t_len = prior_len;
    }
    if (brk || next < 0) break;
    prior = next; prior_off = noff; prior_len = nlen; prior_kind = nkind; prior_full = nfull;
    if (next == 1) nh = F.b(noff);
  }
  E.consumed = p - pos;
  E.rec = E.net_hlen + E.ext_len + E.t_len;
  return true;
}

// The bytes Icmpv4Header / Icmpv6Header::to_bytes write back for an error
// message: only the fields its type defines survive (v4 DestUnreachable code
// 4: the next-hop MTU; Redirect: the gateway; ParameterProblem code 0: the
// pointer byte; v6 PacketTooBig: the MTU; ParameterProblem: the pointer);
// unused bytes -- RFC 4884's length among them -- are zero.
__device__ __forceinline__ void icmp_norm_at(const Frame &F, int o, bool v6) {
  if (!icmp_err_at(F, o, v6)) return;
  const uint8_t t = F.b(o), c = F.b(o + 1);
  if (!v6) {
    if (t == 3) { wput16(F, o + 4, 0); if (c != 4) wput16(F, o + 6, 0); }
    if (t == 11) wput32(F, o + 4, 0);
    if (t == 12) { wput8(F, o + 5, 0); wput16(F, o + 6, 0); if (c != 0) wput8(F, o + 4, 0); }
  } else if (t == 1 || t == 3) {
    wput32(F, o + 4, 0);
  }
}
// An ICMP error message's embedded headers as the deparse writes them back
// (EmbeddedHeaders::deparse): the embedded IPv4 reserved flag bit, extension-header reserved fields, a full
// embedded TCP header's reserved bits and a full embedded ICMP header.
// Applied to the frame right after the parse: every later reader (checksum
// validation, serialize) sees the bytes the reference's structures hold.
__device__ __forceinline__ void emb_normalize(const Frame &F, const Emb &E) {
  if (E.net == 4) wput8(F, E.off + 6, F.b(E.off + 6) & 0x7f);
  for (int e = 0; e < E.next; e++) {
    const int x = E.ext_off[e];
    if (E.ext_kind[e] == HK_EXT_FRAG) { wput8(F, x + 1, 0); wput8(F, x + 3, F.b(x + 3) & 0xf9); }
    if (E.ext_kind[e] == HK_EXT_AUTH) wput16(F, x + 2, 0);
  }
  if (E.full && E.tk == L4_TCP) wput8(F, E.t_off + 12, F.b(E.t_off + 12) & 0xf1);
  if (E.full && (E.tk == L4_ICMP4 || E.tk == L4_ICMP6)) icmp_norm_at(F, E.t_off, E.tk == L4_ICMP6);
}

// What the later stages need of the embedded headers, in one word of the
// parsed header stack: present, IP version and header length, the bytes of
// the kept extension headers (left out of the ICMP checksum), the transport
// kind and whether it is a full header.  Offsets follow from the ICMP
// header's, so they stay right when the serializer moves the stack.
__device__ __forceinline__ uint32_t emb_pack(const Emb &E) {
  return 1u | ((uint32_t)(E.net_hlen >> 2) << 4) | ((uint32_t)E.tk << 10) | ((uint32_t)E.full << 14) |
         ((uint32_t)(E.net == 6) << 15) | ((uint32_t)E.ext_len << 16);
}
struct EmbV { int off, net, net_hlen, t_off, t_len, tk; bool full; };
__device__ __forceinline__ EmbV emb_view(const Frame &F, const Hdr &H) {
  EmbV e;
  e.off = H.l4_off + H.l4_hlen;
  e.net = (H.emb >> 15) & 1 ? 6 : 4;
  e.net_hlen = (int)((H.emb >> 4) & 15) << 2;
  e.tk = (int)((H.emb >> 10) & 7);
  e.full = (H.emb >> 14) & 1;
  e.t_off = e.off + e.net_hlen + (int)(H.emb >> 16);
  if (e.tk == L4_NONE) e.t_len = 0;
  else if (!e.full) e.t_len = F.len - e.t_off;  // a partial header: every remaining byte
  else if (e.tk == L4_TCP) e.t_len = (F.b(e.t_off + 12) >> 4) * 4;
  else if (e.tk == L4_UDP) e.t_len = 8;
  else e.t_len = (e.tk == L4_ICMP4 && (F.b(e.t_off) == 13 || F.b(e.t_off) == 14) && F.b(e.t_off + 1) == 0) ? 20 : 8;
  return e;
}

// The generic loop's result for the dominant shapes -- Ethernet + IPv4 /
// IPv6 without extension headers + UDP (not to the VXLAN port) / TCP --
// computed straight-line; false: not such a frame, run the loop.
__device__ __forceinline__ bool parse_fast(const Frame &F, int hb, Hdr &H) {
  const int pos = hb + 14;
  const int rem = F.len - pos;
  const uint16_t et = F.be16(hb + 12);
  int nhl, proto;
  if (et == 0x0800) {
    if (rem < 20) return false;
    const uint8_t v = F.b(pos);
    nhl = (v & 0xf) * 4;
    if ((v >> 4) != 4 || nhl < 20 || rem < nhl || F.be16(pos + 2) < nhl) return false;
    const uint32_t src = F.be32(pos + 12);
    if ((src >> 28) == 0xe || src == 0xffffffffu) return false;
    proto = F.b(pos + 9);
  } else if (et == 0x86dd) {
    if (rem < 40 || (F.b(pos) >> 4) != 6 || F.b(pos + 8) == 0xff) return false;
    nhl = 40;
    proto = F.b(pos + 6);
  } else {
    return false;
  }
  const int lp = pos + nhl, lrem = F.len - lp;
  int lhl;
  if (proto == 17) {
    if (lrem < 8 || F.be16(lp) == 0 || F.be16(lp + 2) == 0 || F.be16(lp + 2) == 4789) return false;
    lhl = 8;
    H.l4 = L4_UDP;
  } else if (proto == 6) {
    if (lrem < 20) return false;
    lhl = (F.b(lp + 12) >> 4) * 4;
    if (lhl < 20 || lrem < lhl || F.be16(lp) == 0 || F.be16(lp + 2) == 0) return false;
    H.l4 = L4_TCP;
  } else {
    return false;
  }
  H.net = et == 0x0800 ? 4 : 6;
  H.net_off = pos; H.net_hlen = nhl;
  H.l4_off = lp; H.l4_hlen = lhl;
  H.consumed = lp + lhl - hb;
  H.size = 14 + nhl + lhl;
  return true;
}

// Headers::parse (net/src/headers/mod.rs:474-578) incl. the MAX_VLANS /
// MAX_NET_EXTENSIONS quirk.  Returns false if the Ethernet header is invalid.
__device__ __forceinline__ bool parse(const Frame &F, int hb, Hdr &H) {
  H.hb = hb; H.nvlan = 0; H.net = 0; H.next = 0; H.ext_len = 0; H.l4 = L4_NONE;
  H.vx = false; H.vni = 0; H.net_off = H.net_hlen = 0; H.l4_off = H.l4_hlen = 0; H.vx_off = 0;
  H.emb = 0;
  int rem = F.len - hb;
  if (rem < 14) return false;
  uint8_t d0 = 0, s0 = F.b(hb + 6), dz = 0, sz = 0;
  for (int i = 0; i < 6; i++) { uint8_t x = F.b(hb + i); dz |= x; if (i == 0) d0 = x; sz |= F.b(hb + 6 + i); }
  (void)d0;
  if (dz == 0 || sz == 0 || (s0 & 1)) return false;
  if (parse_fast(F, hb, H)) return true;
  H.l4 = L4_NONE;
  int pos = hb + 14;
  bool v6ctx = false;
  uint32_t aux = 0;
  int cur = kind_of_ethertype(F.be16(hb + 12));
  int cur_len = cur ? try_parse(F, cur, pos, aux) : 0;
  if (cur_len == 0) { H.consumed = pos - hb; H.size = 14; return true; }
  int cur_pos = pos;
  uint32_t cur_aux = aux;
  pos += cur_len;
  for (int guard = 0; guard < 16; guard++) {
    // next header from cur's payload
    int nk = HK_NONE;
    switch (cur) {
      case HK_VLAN: nk = kind_of_ethertype(F.be16(cur_pos + 2)); break;
      case HK_V4: nk = kind_of_proto(F.b(cur_pos + 9), false); break;
      case HK_V6: nk = kind_of_proto(F.b(cur_pos + 6), true); break;
      case HK_EXT_RAW: case HK_EXT_FRAG: nk = kind_of_proto(F.b(cur_pos), true); break;
      case HK_EXT_AUTH: {
        uint8_t p = F.b(cur_pos);
        if (v6ctx) nk = kind_of_proto(p, true);
        else nk = (p == 6 || p == 17 || p == 1 || p == 51) ? kind_of_proto(p, false) : HK_NONE;
        break;
      }
      case HK_UDP: nk = F.be16(cur_pos + 2) == 4789 ? HK_VXLAN : HK_NONE; break;
      default: nk = HK_NONE;
    }
    uint32_t naux = 0;
    int nlen = nk ? try_parse(F, nk, pos, naux) : 0;
    int npos = pos;
    if (nlen) pos += nlen;
    bool brk = false;
    switch (cur) {
      case HK_VLAN: if (H.nvlan < 4) H.nvlan++; else brk = true; break;
      case HK_V4: H.net = 4; H.net_off = cur_pos; H.net_hlen = cur_len; v6ctx = false; break;
      case HK_V6: H.net = 6; H.net_off = cur_pos; H.net_hlen = 40; v6ctx = true; break;
      case HK_EXT_RAW: case HK_EXT_FRAG: case HK_EXT_AUTH:
        if (H.next < 3) {
          if (H.next == 0) { H.ext_off[0] = cur_pos; H.ext_kind[0] = (uint8_t)cur; }
          else if (H.next == 1) { H.ext_off[1] = cur_pos; H.ext_kind[1] = (uint8_t)cur; }
          else { H.ext_off[2] = cur_pos; H.ext_kind[2] = (uint8_t)cur; }
          H.ext_len += cur_len;
          H.next++;
        } else brk = true;
        break;
      case HK_TCP: H.l4 = L4_TCP; H.l4_off = cur_pos; H.l4_hlen = cur_len; break;
      case HK_UDP: H.l4 = L4_UDP; H.l4_off = cur_pos; H.l4_hlen = 8; break;
      case HK_ICMP4: H.l4 = L4_ICMP4; H.l4_off = cur_pos; H.l4_hlen = cur_len; break;
      case HK_ICMP6: H.l4 = L4_ICMP6; H.l4_off = cur_pos; H.l4_hlen = cur_len; break;
      case HK_VXLAN: H.vx = true; H.vx_off = cur_pos; H.vni = cur_aux; break;
    }
    if (brk || !nlen) break;
    cur = nk; cur_pos = npos; cur_len = nlen; cur_aux = naux;
  }
  // an ICMP error message's payload: its embedded packet fragment
  // (Icmp4::parse_payload, icmp4/mod.rs:626-646, and the ICMPv6 twin)
  int emb_rec = 0;
  if ((H.l4 == L4_ICMP4 || H.l4 == L4_ICMP6) && pos == H.l4_off + H.l4_hlen &&
      icmp_err_at(F, H.l4_off, H.l4 == L4_ICMP6)) {
    // the header as Icmpv4Header / Icmpv6Header write it back
    icmp_norm_at(F, H.l4_off, H.l4 == L4_ICMP6);
    Emb E;
    if (emb_parse(F, pos, H.l4 == L4_ICMP6, E)) {
      emb_normalize(F, E);
      pos += E.consumed;
      emb_rec = E.rec;
      H.emb = emb_pack(E);
    }
  }
  H.consumed = pos - hb;
  int sz2 = 14 + 4 * H.nvlan;
  if (H.net) {
    sz2 += H.net_hlen + H.ext_len;
    if (H.l4) { sz2 += H.l4_hlen; if (H.vx) sz2 += 8; }
  }
  H.size = sz2 + emb_rec;
  return true;
}

// ---------------------------------------------------------------------------
// Mutable per-packet state (values that differ from the frame bytes)
// ---------------------------------------------------------------------------
struct Addr16 { uint32_t w[4]; };  // network order bytes packed big-endian per word

// VXLAN outer header values (IpForwarder::build_vxlan_headers)
struct OuterHdr {
  uint8_t fam, tos;      // outer IP family; dscp<<2|ecn
  uint16_t sport, len;   // UDP source port; UDP length
  uint32_t vni;
  Addr16 src, dst;
};
// 16-bit words of Eth + outer IP + UDP + VXLAN
__device__ __forceinline__ int outer_words(int fam) { return fam == 4 ? 25 : 35; }
__device__ __forceinline__ uint32_t outer_ck4(const OuterHdr &S);
__device__ __forceinline__ void hput16(LDS_AS uint8_t *o, int i, uint32_t v) { o[i] = (uint8_t)(v >> 8); o[i + 1] = (uint8_t)v; }
__device__ __forceinline__ void hput32(LDS_AS uint8_t *o, int i, uint32_t v) { hput16(o, i, v >> 16); hput16(o, i + 2, v); }

struct State {
  uint8_t done;
  uint32_t flags;
  bool has_vrf;
  uint32_t vrf;
  uint32_t src_vni, dst_vni;
  bool has_oif;
  uint32_t oif;
  uint8_t eg_code, if_code;  // resolved Egress outcome of the last Egress instruction
  uint64_t eg_dmac, eg_smac;
  int32_t fib;           // FIB of `vrf` (precomputed), -1 none
  int32_t vni_idx;       // VniRec of src_vni, -1
  int32_t pair;          // PairRec of (src_vni, dst_vni), -1 unknown
  bool has_dscp;
  uint8_t dscp, ecn;
  uint32_t fib_entry, acl_rule;
  uint8_t acl;
  uint32_t nh_ref;       // PacketMeta.nh_addr source: the last Egress instruction executed
                         // (NH_NONE; bit 31: the single instruction of FibEntry `low bits`)
  // current header field values
  uint64_t edst, esrc;   // current Ethernet dst / src (48-bit, byte 0 on top)
  bool eth_dirty;
  uint8_t ttl;           // v4 ttl / v6 hop limit
  uint32_t v4src, v4dst; // host order
  uint16_t sport, dport;
  // encap
  bool encap;
  uint8_t o_fam;         // outer IP family; the outer IP/UDP/VXLAN headers are
                         // deparsed at encap into the lane's LDS scratch (F.hs)
  bool inner_l4_ck;      // encap: the inner L4 checksum is recomputed
  bool o_eth;            // Egress added the outer Ethernet header
  uint64_t odst, osrc;   // outer Ethernet (encap)
  int pay_start;         // frame-relative payload start (inner after decap)
};

__device__ __forceinline__ void done(State &S, uint8_t r) { if (S.done == DONE_NONE) S.done = r; }
constexpr uint32_t NH_NONE = 0xffffffffu;
constexpr uint32_t NH_ENTRY = 0x80000000u;

__device__ __forceinline__ void load_fields(const Frame &F, const Hdr &H, State &S) {
  S.edst = mac_at(F, H.hb);
  S.esrc = mac_at(F, H.hb + 6);
  S.eth_dirty = false;
  if (H.net == 4) {
    S.ttl = F.b(H.net_off + 8);
    S.v4src = F.be32(H.net_off + 12);
    S.v4dst = F.be32(H.net_off + 16);
  } else if (H.net == 6) {
    S.ttl = F.b(H.net_off + 7);
  }
  if (H.l4 == L4_TCP || H.l4 == L4_UDP) {
    S.sport = F.be16(H.l4_off);
    S.dport = F.be16(H.l4_off + 2);
  } else {
    S.sport = S.dport = 0;
  }
  S.pay_start = H.hb + H.consumed;
}

__device__ __forceinline__ uint8_t net_proto(const Frame &F, const Hdr &H) {
  return H.net == 4 ? F.b(H.net_off + 9) : F.b(H.net_off + 6);
}

__device__ __forceinline__ Addr16 addr16(const Frame &F, int off) {
  Addr16 a;
  for (int i = 0; i < 4; i++) a.w[i] = F.be32(off + 4 * i);
  return a;
}

// current destination address (after NAT) as the LPM key's two 64-bit
// halves (network order, packed big-endian), built in registers: an Addr16
// filled in divergent branches was kept in scratch memory -- a store and a
// reload ahead of every direct-table load
__device__ __forceinline__ void cur_dst_key(const Frame &F, const Hdr &H, const State &S, uint8_t &fam,
                                            uint64_t &khi, uint64_t &klo) {
  auto w32 = [&](int o) {
    return ((uint32_t)F.hs[o] << 24) | ((uint32_t)F.hs[o + 1] << 16) | ((uint32_t)F.hs[o + 2] << 8) | F.hs[o + 3];
  };
  if (S.encap) {
    fam = S.o_fam;
    if (S.o_fam == 4) { khi = (uint64_t)w32(16) << 32; klo = 0; }
    else { khi = ((uint64_t)w32(24) << 32) | w32(28); klo = ((uint64_t)w32(32) << 32) | w32(36); }
    return;
  }
  fam = (uint8_t)H.net;
  if (H.net == 4) { khi = (uint64_t)S.v4dst << 32; klo = 0; return; }
  const int o = H.net_off + 24;
  khi = ((uint64_t)F.be32(o) << 32) | F.be32(o + 4);
  klo = ((uint64_t)F.be32(o + 8) << 32) | F.be32(o + 12);
}

// ---------------------------------------------------------------------------
// rapidhash-style hash (same restatement as the oracle; parity vs the
// reference is UNPINNED)
// ---------------------------------------------------------------------------
struct HBuf { lds_u8 *b; int n; };  // per-thread LDS scratch (no private-array scratch)
__device__ __forceinline__ void hb_put(HBuf &h, uint8_t x) { h.b[h.n++] = x; }
__device__ __forceinline__ void mum(uint64_t &a, uint64_t &b) {
  uint64_t lo = a * b, hi = __umul64hi(a, b);
  a = lo; b = hi;
}
__device__ __forceinline__ uint64_t mixh(uint64_t a, uint64_t b) { mum(a, b); return a ^ b; }
__device__ __forceinline__ uint64_t rd64(const lds_u8 *p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
__device__ __forceinline__ uint64_t rd32(const lds_u8 *p) {
  return (uint64_t)p[0] | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) | ((uint64_t)p[3] << 24);
}
__device__ __forceinline__ uint64_t rapid(const lds_u8 *p, int len) {
  const uint64_t s0 = 0x2d358dccaa6c78a5ull, s1 = 0x8bb84b93962eacc9ull, s2 = 0x4b33a62ed433d4a3ull;
  uint64_t seed = 0xbdd89aa982704029ull;
  seed ^= mixh(seed ^ s0, s1) ^ (uint64_t)len;
  uint64_t a, b;
  if (len <= 16) {
    if (len >= 4) {
      const lds_u8 *pl = p + len - 4;
      a = (rd32(p) << 32) | rd32(pl);
      uint64_t delta = ((uint64_t)(len & 24)) >> (len >> 3);
      b = (rd32(p + delta) << 32) | rd32(pl - delta);
    } else if (len > 0) {
      a = ((uint64_t)p[0] << 56) | ((uint64_t)p[len >> 1] << 32) | p[len - 1];
      b = 0;
    } else {
      a = b = 0;
    }
  } else {
    int i = len;
    if (i > 48) {
      uint64_t see1 = seed, see2 = seed;
      while (i >= 48) {
        seed = mixh(rd64(p) ^ s0, rd64(p + 8) ^ seed);
        see1 = mixh(rd64(p + 16) ^ s1, rd64(p + 24) ^ see1);
        see2 = mixh(rd64(p + 32) ^ s2, rd64(p + 40) ^ see2);
        p += 48;
        i -= 48;
      }
      seed ^= see1 ^ see2;
    }
    if (i > 16) {
      seed = mixh(rd64(p) ^ s2, rd64(p + 8) ^ seed ^ s1);
      if (i > 32) seed = mixh(rd64(p + 16) ^ s2, rd64(p + 24) ^ seed);
    }
    a = rd64(p + i - 16);
    b = rd64(p + i - 8);
  }
  a ^= s1;
  b ^= seed;
  mum(a, b);
  return mixh(a ^ s0 ^ (uint64_t)len, b ^ s1);
}

// The stream is what the reference's Hasher calls feed it, in order
// (net/src/packet/hash.rs:17-68; DESIGN.md §4 lists each field's Hash):
// every write_uN(v) as v's native (little-endian) bytes -- the Hasher
// trait's default encoding -- a slice's length prefix as write_usize.  An
// address's Hash is write_u32 / write_u128 of u32 / u128::from_ne_bytes(octets),
// so its bytes are the octets in network order.
__device__ __forceinline__ void hb_u16(HBuf &h, uint32_t v) { hb_put(h, (uint8_t)v); hb_put(h, (uint8_t)(v >> 8)); }
__device__ __forceinline__ void hb_usize(HBuf &h, uint32_t v) {
  hb_u16(h, v); hb_u16(h, 0); hb_u16(h, 0); hb_u16(h, 0);
}
__device__ __forceinline__ void hash_ip_fields(const Frame &F, const Hdr &H, const State &S, HBuf &h) {
  if (H.net == 4) {
    for (int i = 0; i < 4; i++) hb_put(h, (uint8_t)(S.v4src >> (24 - 8 * i)));  // source(): write_u32
    for (int i = 0; i < 4; i++) hb_put(h, (uint8_t)(S.v4dst >> (24 - 8 * i)));  // destination(): write_u32
    hb_put(h, F.b(H.net_off + 9));                                              // protocol(): write_u8
  } else if (H.net == 6) {
    for (int i = 0; i < 32; i++) hb_put(h, F.b(H.net_off + 8 + i));            // write_u128 x 2
    hb_put(h, F.b(H.net_off + 6));                                              // next_header(): write_u8
  } else {
    return;
  }
  if (H.l4 == L4_TCP || H.l4 == L4_UDP) {  // TcpPort / UdpPort: write_u16 each
    hb_u16(h, S.sport);
    hb_u16(h, S.dport);
  } else if (H.l4 == L4_ICMP4 || H.l4 == L4_ICMP6) {
    uint8_t t = F.b(H.l4_off);
    bool echo = H.l4 == L4_ICMP4 ? (t == 0 || t == 8) : (t == 128 || t == 129);
    if (echo) hb_u16(h, ((uint32_t)F.b(H.l4_off + 4) << 8) | F.b(H.l4_off + 5));  // identifier(): write_u16
  }
}

// ---------------------------------------------------------------------------
// LPM (Poptrie-style, see dp_tables.cpp build_poptrie)
// ---------------------------------------------------------------------------
// 6 bits of the key at [off, off+6), zero-padded past the address width
// (v4 keys carry zeros in w[1..3]); the key is held as two u64 halves.
// bits [off, off + 6) of the 128-bit key (hi:lo), zero past bit 127 -- selects, no branches
__device__ __forceinline__ uint32_t key6(uint64_t hi, uint64_t lo, int off) {
  const int o = off & 63;
  uint64_t x = off < 64 ? (hi << o) | ((lo >> 1) >> (63 - o)) : lo << o;
  if (off >= 128) x = 0;
  return (uint32_t)(x >> 58);
}

// sel = off | shift << 8 | bits << 16: the first table is indexed by `bits`
// key bits taken at (khi >> shift), and the Poptrie below it starts at key bit
// `off` -- the direct table (bits = off = dbits, shift = 64 - dbits) or a v6
// FIB's window table (Lpm.wtab: the wtb bits after the window's shared prefix)
__device__ __forceinline__ uint32_t lpm_sel(uint32_t off, uint32_t shift, uint32_t bits) {
  return off | (shift << 8) | (bits << 16);
}
// the selector of an Lpm's direct table (its dbits, DPD_LPM_D16 in bit 24)
__device__ __forceinline__ uint32_t lpm_dsel(uint32_t dbits) {
  const uint32_t b = dbits & 0xffu;
  return lpm_sel(b, 64 - b, b) | ((dbits & DPD_LPM_D16) << 16);
}
__device__ __forceinline__ uint32_t lpm_walk(const Img &g, uint64_t table_off, uint32_t sel, uint64_t blocks,
                                             uint64_t khi, uint64_t klo) {
  const uint32_t w0 = (uint32_t)(khi >> 32);
  int off = (int)(sel & 0xffu);
  if (sel >> 24) {  // DIR-24-8 with 16-bit direct entries (v4)
    const uint32_t e = g.at<uint16_t>(table_off)[w0 >> 8];
    TRIP();
    if (e & 0x8000u) return e & 0x7fffu;
    TRIP();
    return g.at<uint16_t>(blocks)[(e << 8) | (w0 & 0xff)];
  }
#if DP_V6W
  const uint32_t e = g.at<uint32_t>(table_off)[(uint32_t)(khi >> ((sel >> 8) & 0xffu)) &
                                               ((1u << ((sel >> 16) & 0xffu)) - 1u)];
#else
  const uint32_t e = g.at<uint32_t>(table_off)[w0 >> (32 - off)];  // the direct table (dbits <= 32)
#endif
  TRIP();
  if (e & 0x80000000u) return e & 0x7fffffffu;
  TRIP();
  if (blocks) return g.at<uint16_t>(blocks)[(e << 8) | (w0 & 0xff)];  // DIR-24-8 (v4)
  const PtNode *nodes = g.at<PtNode>(g.im.pt_nodes);
  const uint32_t *leaves = g.at<uint32_t>(g.im.pt_leaves);
  uint32_t ni = e;
  for (int guard = 0; guard < 24; guard++) {
    const PtNode &nd = nodes[ni];
    TRIP();
    uint64_t vec = nd.vec, lv = nd.leafvec;
    uint32_t v = key6(khi, klo, off);
    uint64_t bit = 1ull << v;
    if (vec & bit) {
      ni = nd.base1 + (uint32_t)__popcll(vec & (bit - 1));
      off += 6;
      continue;
    }
    uint64_t m = (v == 63) ? ~0ull : ((bit << 1) - 1);
    return leaves[nd.base0 + (uint32_t)__popcll(lv & m) - 1];
  }
  return g.im.drop_nh;  // unreachable for a well-formed image
}
__device__ __forceinline__ uint32_t lpm_lookup(const Img &g, const Lpm &L, const Addr16 &a) {
  const uint64_t khi = ((uint64_t)a.w[0] << 32) | a.w[1], klo = ((uint64_t)a.w[2] << 32) | a.w[3];
  if (DP_V6W && L.wtab && (khi >> (64 - L.wbits)) == L.wpfx)
    return lpm_walk(g, L.wtab, lpm_sel(L.wbits + L.wtb, 64 - L.wbits - L.wtb, L.wtb), 0, khi, klo);
  return lpm_walk(g, L.direct, lpm_dsel(L.dbits), L.blocks, khi, klo);
}

// Multibit index walk from a context record's descriptor (Mbi): leaf value
// (DPD_LEAF stripped) of `key` (an address, or a port with kbits 16).
__device__ __forceinline__ uint32_t mbi_walk(const Img &g, const Mbi &m, uint32_t key) {
  const int rem0 = (int)m.kbits - (int)m.s0;
  uint32_t e = g.at<uint32_t>(m.root)[key >> rem0];
  TRIP();
#pragma unroll
  for (int l = 1; l <= 3; l++)
    if (!(e & DPD_LEAF) && (TRIP(), true)) e = g.at<uint32_t>(m.blocks)[(e << 8) | ((key >> (rem0 - 8 * l)) & 0xff)];
  return e & ~DPD_LEAF;
}

// ---------------------------------------------------------------------------
// Classifier (bit-vector, first match)
// ---------------------------------------------------------------------------
struct Key128 { uint64_t hi, lo; };

// field of the v4 ([0]) or v6 ([1]) classifier; a select, never a dynamic
// index into the kernel-argument image header (which would force a private copy)
#define CLS(arr, t, field) ((t) ? g.im.arr[1].field : g.im.arr[0].field)

// The bounds range [lo, hi) a field's jump table leaves for a key: its
// 16-bit bucket's (v4 address >> 16, port, v6 address >> 112).
__device__ __forceinline__ void jump_range(const uint32_t *jt, const FieldIdx &f, Key128 k, uint32_t &lo,
                                           uint32_t &hi) {
  const uint32_t b = f.shift == 48 ? (uint32_t)(k.hi >> 48) : (uint32_t)(k.lo >> f.shift) & 0xffff;
  lo = jt[b];
  hi = jt[b + 1] + 1;
}

// A v6 address key in the space of the classifiers' v6 indexes (Image.v6w_*):
// the rules of one site share their top bits, so the indexes order the bits
// after them (a top-16-bit jump table would hold every rule in one bucket).
// Image-wide and uniform: the window test is one compare per key.
__device__ __forceinline__ Key128 v6_window_key(uint32_t c, uint64_t p, Key128 k) {
  if (!c) return k;
  const uint64_t top = k.hi >> (64 - c);
  if (top != p) return top < p ? Key128{0, 0} : Key128{~0ull, ~0ull};
  return Key128{(k.hi << c) | (k.lo >> (64 - c)), (k.lo << c) | 1};
}

// Elementary interval of one key in one field index -> its leaf value
// (bit-vector row id, or packed candidate run).
__device__ __forceinline__ uint32_t field_leaf(const Img &g, const FieldIdx &F, Key128 key) {
  if (F.root) {
    uint32_t k = (uint32_t)key.lo;
    uint32_t e = g.at<uint32_t>(F.root)[k >> (F.kbits - F.s0)];
    TRIP();
#pragma unroll
    for (int l = 1; l <= 3; l++) {
      if (!(e & DPD_LEAF)) {
        TRIP();
        int rem = (int)F.kbits - (int)F.s0 - 8 * l;
        e = g.at<uint32_t>(F.blocks)[(e << 8) | ((k >> rem) & 0xff)];
      }
    }
    return e & ~DPD_LEAF;
  }
  if (DP_V6W && F.shift == 48) key = v6_window_key(g.im.v6w_c, g.im.v6w_p, key);  // a v6 address field
  uint32_t lo = 0, hi = F.n;
  if (F.jump) jump_range(g.at<uint32_t>(F.jump), F, key, lo, hi);
  const uint64_t *bd = g.at<uint64_t>(F.bounds);
  while (hi - lo > 1) {
    TRIP();
    uint32_t mid = (lo + hi) >> 1;
    uint64_t bh = bd[2 * (uint64_t)mid], bl = bd[2 * (uint64_t)mid + 1];
    bool le = bh < key.hi || (bh == key.hi && bl <= key.lo);
    if (le) lo = mid; else hi = mid;
  }
  return g.at<uint32_t>(F.rows)[lo];
}

// key inside the prefix (network a, length len) -- v4 keys use lo only
__device__ __forceinline__ bool pfx_ok(Key128 k, uint64_t ahi, uint64_t alo, uint32_t len, bool v6) {
  if (len == 0) return true;
  if (!v6) return (((uint32_t)k.lo ^ (uint32_t)alo) >> (32 - len)) == 0;
  if (len <= 64) return ((k.hi ^ ahi) >> (64 - len)) == 0;
  if (k.hi != ahi) return false;
  return len == 128 ? k.lo == alo : ((k.lo ^ alo) >> (128 - len)) == 0;
}

// Bit-vector group: global rule index of the first match, or -1.  Kept out
// of line: its lockstep state is large and the candidate-list form is the
// common one.  Every argument is a value or a pointer into the table image
// (global memory): nothing of the caller's private frame or LDS crosses the
// call (DESIGN.md "Out-of-line device functions").
__device__ DP_BV int64_t classify_bv(const uint8_t *base, const Group *Gp, uint8_t proto, Key128 src,
                                       Key128 dst, uint16_t sp, uint16_t dp, uint32_t wc, uint64_t wp) {
  const ImgBase g{base};
  const Group G = *Gp;
  Key128 key[4] = {src, dst, Key128{0, sp}, Key128{0, dp}};
  // v6 address fields index the window's key space (v6_window_key)
  if (DP_V6W && G.f[0].shift == 48) key[0] = v6_window_key(wc, wp, key[0]);
  if (DP_V6W && G.f[1].shift == 48) key[1] = v6_window_key(wc, wp, key[1]);
  uint32_t lo[4], hi[4], e[4];
  // level 0 of every field: multibit root entry, or the jump-table range
#pragma unroll
  for (int f = 0; f < 4; f++) {
    lo[f] = 0;
    hi[f] = G.f[f].n;
    e[f] = DPD_LEAF;
    if (G.f[f].root) {
      uint32_t k = (uint32_t)key[f].lo;
      e[f] = g.at<uint32_t>(G.f[f].root)[k >> (G.f[f].kbits - G.f[f].s0)];
      hi[f] = lo[f] + 1;  // no bounds search
    } else if (G.f[f].jump) {
      jump_range(g.at<uint32_t>(G.f[f].jump), G.f[f], key[f], lo[f], hi[f]);
    }
  }
  // multibit levels (8 bits each), in lockstep
#pragma unroll
  for (int l = 1; l <= 3; l++) {
#pragma unroll
    for (int f = 0; f < 4; f++) {
      if (!(e[f] & DPD_LEAF)) {
        int rem = (int)G.f[f].kbits - (int)G.f[f].s0 - 8 * l;
        uint32_t k = (uint32_t)key[f].lo;
        e[f] = g.at<uint32_t>(G.f[f].blocks)[(e[f] << 8) | ((k >> rem) & 0xff)];
      }
    }
  }
  // bounds form: binary search in lockstep
  for (int it = 0; it < 20; it++) {
    bool any = false;
#pragma unroll
    for (int f = 0; f < 4; f++) {
      if (hi[f] - lo[f] > 1) {
        uint32_t mid = (lo[f] + hi[f]) >> 1;
        const uint64_t *b = g.at<uint64_t>(G.f[f].bounds) + 2 * (uint64_t)mid;
        uint64_t bh = b[0], bl = b[1];
        bool le = bh < key[f].hi || (bh == key[f].hi && bl <= key[f].lo);
        if (le) lo[f] = mid; else hi[f] = mid;
        any = true;
      }
    }
    if (!any) break;
  }
  uint32_t rr[4];
#pragma unroll
  for (int f = 0; f < 4; f++)
    rr[f] = G.f[f].root ? (e[f] & ~DPD_LEAF) : g.at<uint32_t>(G.f[f].rows)[lo[f]];
  const uint64_t *pool = g.at<uint64_t>(G.pool);
  uint32_t stride = G.sum_words + G.words;
  uint32_t r0 = g.at<uint16_t>(G.proto_rows)[proto];
  uint32_t r1 = rr[0], r2 = rr[1], r3 = rr[2], r4 = rr[3];
  const uint64_t *p0 = pool + (uint64_t)r0 * stride, *p1 = pool + (uint64_t)r1 * stride;
  const uint64_t *p2 = pool + (uint64_t)r2 * stride, *p3 = pool + (uint64_t)r3 * stride;
  const uint64_t *p4 = pool + (uint64_t)r4 * stride;
  int64_t ri = -1;
  for (uint32_t s = 0; s < G.sum_words && ri < 0; s++) {
    uint64_t m = p0[s] & p1[s] & p2[s] & p3[s] & p4[s];
    while (m) {
      uint32_t w = s * 64 + (uint32_t)__ffsll((unsigned long long)m) - 1;
      uint32_t o = G.sum_words + w;
      uint64_t x = p0[o] & p1[o] & p2[o] & p3[o] & p4[o];
      if (x) { ri = (int64_t)G.rule_base + (int64_t)w * 64 + (__ffsll((unsigned long long)x) - 1); break; }
      m &= m - 1;
    }
  }
  return ri;
}

// Classification result: global rule index (-1: no match) and the rule's
// action words (inline in the candidate record, else from the arrays).
struct Hit {
  int64_t rule;
  uint32_t action, action2, aux, orig;
};
struct ClsArrays { uint64_t group_recs, action, action2, aux, orig, recs; };
#define CLS_ARRAYS(arr, t) ClsArrays{CLS(arr, t, group_recs), CLS(arr, t, action), CLS(arr, t, action2), CLS(arr, t, aux), CLS(arr, t, orig), CLS(arr, t, recs)}
// no hoisted index leaf (see hoist_walks)
constexpr uint32_t NO_PRE = 0xffffffffu;
enum { W_ACTION = 1, W_ACTION2 = 2, W_AUX = 4, W_ORIG = 8 };

// First match of (proto, src, dst, sport, dport) in group gi.
//  - candidate-list groups: index of one field -> verify the inline
//    candidates in precedence order;
//  - bit-vector groups: the four field searches (elementary interval
//    containing the key) run in lockstep so their loads overlap, then the
//    rows are ANDed behind the summary level; first set bit wins.
__device__ __forceinline__ Hit verify_run(const Img &g, uint64_t recs, uint32_t run, bool v6, uint8_t proto,
                                          Key128 src, Key128 dst, uint16_t sp, uint16_t dp, bool acl = false) {
  Hit h{-1, 0, 0, 0, 0};
  const uint32_t first = run >> DPD_RUN_BITS, cnt = run & DPD_RUN_MAX;
  if (!v6) {
    // v4: 32-byte records (CandRec4), DP_CAND4 candidates per round trip --
    // their 16-byte words are requested together
    const uint4 *R = g.at<uint4>(recs) + 2 * (uint64_t)first;
    const uint32_t s = (uint32_t)src.lo, d = (uint32_t)dst.lo;
    auto match4 = [&](const uint4 &w0, const uint4 &w1) -> bool {
      const uint32_t slen = w0.z & 0xff, dlen = (w0.z >> 8) & 0xff;
      const uint32_t pval = (w0.z >> 16) & 0xff, pmask = w0.z >> 24;
      if ((proto & pmask) != (pval & pmask)) return false;
      if (sp < (w0.w & 0xffff) || sp > (w0.w >> 16) || dp < (w1.x & 0xffff) || dp > (w1.x >> 16)) return false;
      if (slen && ((s ^ w0.x) >> (32 - slen))) return false;
      if (dlen && ((d ^ w0.y) >> (32 - dlen))) return false;
      return true;
    };
#pragma unroll 1
    for (uint32_t c = 0; c < cnt; c += DP_CAND4) {
      TRIP();
      if (acl) GTRIP(14); else GTRIP(13);
      // named registers, not an array: a dynamically indexed array would live in scratch
      const uint4 z = make_uint4(0, 0, 0, 0);
      const uint4 *q = R + 2 * c;
      const uint4 a0 = q[0], a1 = q[1];
      const uint4 b0 = c + 1 < cnt ? q[2] : z, b1 = c + 1 < cnt ? q[3] : z;
#if DP_CAND4 == 4
      const uint4 c0 = c + 2 < cnt ? q[4] : z, c1 = c + 2 < cnt ? q[5] : z;
      const uint4 d0 = c + 3 < cnt ? q[6] : z, d1 = c + 3 < cnt ? q[7] : z;
#endif
      uint4 hit = z;
      bool found = true;
      if (match4(a0, a1)) hit = a1;
      else if (c + 1 < cnt && match4(b0, b1)) hit = b1;
#if DP_CAND4 == 4
      else if (c + 2 < cnt && match4(c0, c1)) hit = c1;
      else if (c + 3 < cnt && match4(d0, d1)) hit = d1;
#endif
      else found = false;
      if (found) {
        h.rule = hit.w; h.action = hit.y; h.action2 = hit.z; h.orig = hit.z; h.aux = hit.w;
        return h;
      }
    }
    return h;
  }
  // v6: four 16-byte words per record: src, dst, (lens, proto, ports, rule),
  // (action, action2, aux, orig); every word of a candidate is requested at
  // once and candidates come two per round trip
  const uint4 *R = g.at<uint4>(recs) + 4 * (uint64_t)first;
  auto match = [&](const uint4 &w0, const uint4 &w1, const uint4 &w2) -> bool {
    const uint32_t slen = w2.x & 0xff, dlen = (w2.x >> 8) & 0xff;
    const uint32_t pval = (w2.x >> 16) & 0xff, pmask = w2.x >> 24;
    if ((proto & pmask) != (pval & pmask)) return false;
    if (sp < (w2.y & 0xffff) || sp > (w2.y >> 16) || dp < (w2.z & 0xffff) || dp > (w2.z >> 16)) return false;
    const uint64_t shi = ((uint64_t)w0.y << 32) | w0.x, slo = ((uint64_t)w0.w << 32) | w0.z;
    const uint64_t dhi = ((uint64_t)w1.y << 32) | w1.x, dlo = ((uint64_t)w1.w << 32) | w1.z;
    return pfx_ok(src, shi, slo, slen, v6) && pfx_ok(dst, dhi, dlo, dlen, v6);
  };
#pragma unroll 1
  for (uint32_t c = 0; c < cnt; c += 2) {
    TRIP();
    const uint4 *a = R + 4 * c;
    const uint4 a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
    uint4 b0 = make_uint4(0, 0, 0, 0), b1 = b0, b2 = make_uint4(0, 0, 0, 0), b3 = b0;
    const bool two = c + 1 < cnt;
    if (two) { b0 = a[4]; b1 = a[5]; b2 = a[6]; b3 = a[7]; }
    if (match(a0, a1, a2)) {
      h.rule = a2.w; h.action = a3.x; h.action2 = a3.y; h.aux = a3.z; h.orig = a3.w;
      return h;
    }
    if (two && match(b0, b1, b2)) {
      h.rule = b2.w; h.action = b3.x; h.action2 = b3.y; h.aux = b3.z; h.orig = b3.w;
      return h;
    }
  }
  return h;
}

// `pre`: the group's list-index leaf when hoist_walks already walked it.
template <int WANT>
__device__ __forceinline__ Hit classify(const Img &g, const ClsArrays &A, int32_t gi, bool v6,
                                        uint8_t proto, Key128 src, Key128 dst, uint16_t sp, uint16_t dp,
                                        uint32_t pre = NO_PRE) {
  Hit h{-1, 0, 0, 0, 0};
  if (gi < 0) return h;
  if (pre != NO_PRE) { GTRIP(15); return verify_run(g, A.recs, pre, v6, proto, src, dst, sp, dp, (WANT & W_ORIG) != 0); }
  const Group *Gp = g.at<Group>(A.group_recs) + gi;
  if (Gp->mode == DPD_GROUP_LIST) {
    const uint32_t f = Gp->lfield;
    const FieldIdx F = Gp->f[f];
    Key128 k = f == 0 ? src : f == 1 ? dst : Key128{0, f == 2 ? sp : dp};
    GTRIP(12);
    return verify_run(g, A.recs, field_leaf(g, F, k), v6, proto, src, dst, sp, dp, (WANT & W_ORIG) != 0);
  }
  const int64_t ri = classify_bv(g.base, Gp, proto, src, dst, sp, dp, g.im.v6w_c, g.im.v6w_p);
  if (ri < 0) return h;
  h.rule = ri;
  if (WANT & W_ACTION) h.action = g.at<uint32_t>(A.action)[ri];
  if (WANT & W_ACTION2) h.action2 = g.at<uint32_t>(A.action2)[ri];
  if (WANT & W_AUX) h.aux = g.at<uint32_t>(A.aux)[ri];
  if (WANT & W_ORIG) h.orig = g.at<uint32_t>(A.orig)[ri];
  return h;
}

// ---------------------------------------------------------------------------
// Static NAT
// ---------------------------------------------------------------------------
// Two lookups (src table, dst table) in lockstep so their dependent loads
// overlap.  Per lookup: q.ti table (-1: none), q.addr, q.port.  Result:
// ok, new address, has_new_port, new port.
struct NatQ {
  int32_t ti;
  uint32_t addr;
  uint16_t port;
  bool ok, hp;
  uint32_t na;
  uint16_t np;
};

// the entry's j-th port range (packed lo | hi << 16): inline for one range
__device__ __forceinline__ uint32_t nat_pr(const NatEnt &E, const uint32_t *prs, uint32_t j) {
  return (E.inl & 2) ? E.first_pr : prs[E.first_pr + j];
}
__device__ __forceinline__ void nat_find2(const Img &g, NatQ q[2], bool has_port, const uint32_t pre[2]) {
  const NatTab *tabs = g.at<NatTab>(g.im.nat_tab_recs);
  const NatEnt *ents = g.at<NatEnt>(g.im.nat_ents);
  const uint32_t *prs = g.at<uint32_t>(g.im.nat_prs);
  const NatRange *ranges = g.at<NatRange>(g.im.nat_ranges);
  NatTab T[2];
  uint32_t e[2], lo[2], hi[2];
  int32_t ei[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    q[k].ok = false; q[k].hp = false; q[k].na = 0; q[k].np = 0;
    ei[k] = -1; e[k] = DPD_LEAF; lo[k] = 0; hi[k] = 0;
    if (q[k].ti >= 0 && pre[k] != NO_PRE) {
      e[k] = DPD_LEAF | pre[k];       // multibit walk done by hoist_walks
      T[k].root = 1; T[k].n = 1;
    } else if (q[k].ti >= 0) {
      TRIP();
      T[k] = tabs[q[k].ti];
      if (T[k].root) e[k] = g.at<uint32_t>(T[k].root)[q[k].addr >> (32 - T[k].s0)];
      else hi[k] = T[k].n;
    }
  }
  // multibit levels / small bounds search
  if ((!(e[0] & DPD_LEAF) && q[0].ti >= 0) || (!(e[1] & DPD_LEAF) && q[1].ti >= 0)) TRIP();
#pragma unroll
  for (int l = 1; l <= 3; l++) {
    if (!(e[0] & DPD_LEAF) || !(e[1] & DPD_LEAF)) TRIP();
#pragma unroll
    for (int k = 0; k < 2; k++)
      if (!(e[k] & DPD_LEAF))
        e[k] = g.at<uint32_t>(T[k].blocks)[(e[k] << 8) | ((q[k].addr >> (32 - T[k].s0 - 8 * l)) & 0xff)];
  }
  for (int it = 0; it < 8; it++) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < 2; k++)
      if (hi[k] - lo[k] > 1) {
        uint32_t mid = (lo[k] + hi[k]) >> 1;
        if (g.at<uint32_t>(T[k].bounds)[mid] <= q[k].addr) lo[k] = mid; else hi[k] = mid;
        any = true;
      }
    if (!any) break;
    TRIP();
  }
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (q[k].ti < 0 || T[k].n == 0) continue;
    ei[k] = T[k].root ? (int32_t)(e[k] & ~DPD_LEAF) - 1 : g.at<int32_t>(T[k].longest)[lo[k]];
  }
  // IpPortPrefixTrie::lookup: longest matching prefix whose port set covers
  NatEnt E[2];
  bool fin[2] = {false, false};
  for (int it = 0; it < 33; it++) {
    bool any = false;
    if ((ei[0] >= 0 && !fin[0]) || (ei[1] >= 0 && !fin[1])) TRIP();
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (ei[k] < 0 || fin[k]) continue;
      E[k] = ents[ei[k]];
      bool cov = false;
      if (has_port) {
        if (!E[k].is_pat) cov = true;
        else
          for (uint32_t j = 0; j < E[k].n_pr; j++) {
            uint32_t pr = nat_pr(E[k], prs, j);
            if ((pr & 0xffff) <= q[k].port && q[k].port <= (pr >> 16)) { cov = true; break; }
          }
      }
      if (cov || E[k].covers_all) fin[k] = true;
      else ei[k] = E[k].parent;
      any = true;
    }
    if (!any) break;
  }
  // range of the entry (DisjointRangesBTreeMap::lookup) and the mapping
  uint32_t rl[2], rh[2];
  uint64_t eo[2];
  uint32_t prlo[2];
  bool live[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    live[k] = ei[k] >= 0;
    rl[k] = 0; rh[k] = 0; eo[k] = 0; prlo[k] = 0;
    if (!live[k]) continue;
    if (E[k].is_pat) TRIP();
    const uint32_t addr = q[k].addr;
    const uint64_t ip_off = (uint64_t)(addr - E[k].net);
    const uint64_t esize = ((uint64_t)E[k].size_hi << 32) | E[k].size_lo;
    if (!E[k].is_pat) {
      if (ip_off >= esize) { live[k] = false; continue; }
      eo[k] = ip_off;
    } else {
      if (!has_port) { live[k] = false; continue; }
      int pk = -1;
      for (uint32_t j = 0; j < E[k].n_pr; j++) {
        uint32_t pr = nat_pr(E[k], prs, j);
        if ((pr & 0xffff) <= q[k].port && q[k].port <= (pr >> 16)) { pk = (int)j; break; }
      }
      if (pk < 0) { live[k] = false; continue; }
      uint32_t pr = nat_pr(E[k], prs, (uint32_t)pk);
      uint64_t plen = (uint64_t)(pr >> 16) - (pr & 0xffff) + 1;
      eo[k] = ip_off * plen + (uint64_t)(q[k].port - (pr & 0xffff));
      if (eo[k] >= esize) { live[k] = false; continue; }
    }
    if (E[k].inl & 1) {
      // the only range is inline in the entry: no search
      const bool le = E[k].is_pat ? (E[k].olo_ip < addr || (E[k].olo_ip == addr && E[k].olo_port <= q[k].port))
                                  : E[k].olo_ip <= addr;
      rl[k] = rh[k] = le ? 1u : 0u;
    } else {
      rh[k] = E[k].n_ranges;
    }
  }
  for (int it = 0; it < 32; it++) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (!live[k] || rl[k] >= rh[k]) continue;
      if (k == 0 || !(live[0] && rl[0] < rh[0])) TRIP();
      uint32_t m = (rl[k] + rh[k]) >> 1;
      const NatRange &R = ranges[E[k].first_range + m];
      bool le = E[k].is_pat ? (R.olo_ip < q[k].addr || (R.olo_ip == q[k].addr && R.olo_port <= q[k].port))
                            : R.olo_ip <= q[k].addr;
      if (le) rl[k] = m + 1; else rh[k] = m;
      any = true;
    }
    if (!any) break;
  }
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (!live[k]) continue;
    int sel = (int)rl[k] - 1;
    if (sel < 0) continue;
    NatRange R;
    if (E[k].inl & 1) {
      R.olo_ip = E[k].olo_ip; R.ohi_ip = E[k].ohi_ip; R.olo_port = E[k].olo_port; R.ohi_port = E[k].ohi_port;
      R.tlo_ip = E[k].tlo_ip; R.thi_ip = E[k].thi_ip; R.tlo_port = E[k].tlo_port; R.thi_port = E[k].thi_port;
      R.offset = E[k].offset;
    } else {
      TRIP();
      R = ranges[E[k].first_range + sel];
    }
    const uint32_t addr = q[k].addr;
    if (!E[k].is_pat) {
      if (addr > R.ohi_ip) continue;
      uint64_t o2 = eo[k] - R.offset;
      uint64_t tl = (uint64_t)R.thi_ip - R.tlo_ip + 1;
      if (o2 >= tl) continue;
      q[k].na = R.tlo_ip + (uint32_t)o2;
      q[k].ok = true;
    } else {
      if (addr > R.ohi_ip || (addr == R.ohi_ip && q[k].port > R.ohi_port)) continue;
      uint64_t o2 = eo[k] - R.offset;
      uint64_t tpl = (uint64_t)R.thi_port - R.tlo_port + 1;
      uint64_t tip = (uint64_t)R.thi_ip - R.tlo_ip + 1;
      if (o2 >= tip * tpl) continue;
      // o2 / tpl, o2 % tpl (tpl <= 65536): 32-bit division unless o2 needs more
      uint64_t dq;
      if (!(o2 >> 32)) dq = (uint32_t)o2 / (uint32_t)tpl;
      else dq = o2 / tpl;
      uint16_t np = (uint16_t)(R.tlo_port + (o2 - dq * tpl));
      if (np == 0) continue;
      q[k].na = R.tlo_ip + (uint32_t)dq;
      q[k].np = np;
      q[k].hp = true;
      q[k].ok = true;
    }
  }
}

// ---------------------------------------------------------------------------
// One's complement sums
// ---------------------------------------------------------------------------
// one's complement fold of a 64-bit sum to 16 bits (fixed steps, no loop:
// <= 2^33 after the first, <= 0x2fffe, <= 0x10001, <= 0xffff)
__device__ __forceinline__ uint32_t fold(uint64_t s) {
  s = (s & 0xffffffffull) + (s >> 32);
  uint32_t v = (uint32_t)(s & 0xffff) + (uint32_t)(s >> 16);
  v = (v & 0xffff) + (v >> 16);
  v = (v & 0xffff) + (v >> 16);
  return v;
}
__device__ __forceinline__ uint16_t bswap16(uint32_t v) { return (uint16_t)(((v & 0xff) << 8) | ((v >> 8) & 0xff)); }

// Sum of the big-endian 16-bit words of frame bytes [a, e) (word pairing
// starts at a), returned folded (not complemented).
__device__ __forceinline__ uint32_t sum_frame(const Frame &F, int a, int e) {
  if (e <= a) return 0;
  // absolute alignment: the LDS window starts 16-aligned, frame byte f sits
  // at window position shift + f, which has the same alignment as HBM.
  int wa = F.shift + a, we = F.shift + e;  // window coordinates
  int d0 = wa & ~3, d1 = (we + 3) & ~3;
  uint64_t s = 0;
  const uint8_t *gbase = F.g - F.shift;  // 16-aligned HBM address of window pos 0
  auto masked = [&](uint32_t x, int dd) -> uint32_t {
    if (dd < wa) x &= 0xffffffffu << (8 * (wa - dd));
    if (dd + 4 > we) x &= 0xffffffffu >> (8 * (dd + 4 - we));
    return x;
  };
  int d = d0;
  while (d < d1) {
    if (F.inwin || d + 4 <= WIN) {
      s += masked(*reinterpret_cast<const lds_u32 *>(F.lds + d), d);
      d += 4;
    } else if ((d & 15) == 0 && d + 128 <= d1) {
      // beyond the window: 128 bytes per round trip (eight 16-byte loads
      // issued together), not one load waited on per iteration
      const uint4 *q = reinterpret_cast<const uint4 *>(gbase + d);
      const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4], q5 = q[5], q6 = q[6], q7 = q[7];
      s += (uint64_t)masked(q0.x, d) + masked(q0.y, d + 4) + masked(q0.z, d + 8) + masked(q0.w, d + 12);
      s += (uint64_t)masked(q1.x, d + 16) + masked(q1.y, d + 20) + masked(q1.z, d + 24) + masked(q1.w, d + 28);
      s += (uint64_t)masked(q2.x, d + 32) + masked(q2.y, d + 36) + masked(q2.z, d + 40) + masked(q2.w, d + 44);
      s += (uint64_t)masked(q3.x, d + 48) + masked(q3.y, d + 52) + masked(q3.z, d + 56) + masked(q3.w, d + 60);
      s += (uint64_t)masked(q4.x, d + 64) + masked(q4.y, d + 68) + masked(q4.z, d + 72) + masked(q4.w, d + 76);
      s += (uint64_t)masked(q5.x, d + 80) + masked(q5.y, d + 84) + masked(q5.z, d + 88) + masked(q5.w, d + 92);
      s += (uint64_t)masked(q6.x, d + 96) + masked(q6.y, d + 100) + masked(q6.z, d + 104) + masked(q6.w, d + 108);
      s += (uint64_t)masked(q7.x, d + 112) + masked(q7.y, d + 116) + masked(q7.z, d + 120) + masked(q7.w, d + 124);
      d += 128;
    } else if ((d & 15) == 0 && d + 64 <= d1) {
      const uint4 *q = reinterpret_cast<const uint4 *>(gbase + d);
      const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
      s += (uint64_t)masked(q0.x, d) + masked(q0.y, d + 4) + masked(q0.z, d + 8) + masked(q0.w, d + 12);
      s += (uint64_t)masked(q1.x, d + 16) + masked(q1.y, d + 20) + masked(q1.z, d + 24) + masked(q1.w, d + 28);
      s += (uint64_t)masked(q2.x, d + 32) + masked(q2.y, d + 36) + masked(q2.z, d + 40) + masked(q2.w, d + 44);
      s += (uint64_t)masked(q3.x, d + 48) + masked(q3.y, d + 52) + masked(q3.z, d + 56) + masked(q3.w, d + 60);
      d += 64;
    } else if ((d & 15) == 0 && d + 16 <= d1) {
      const uint4 q = *reinterpret_cast<const uint4 *>(gbase + d);
      s += (uint64_t)masked(q.x, d) + masked(q.y, d + 4) + masked(q.z, d + 8) + masked(q.w, d + 12);
      d += 16;
    } else {
      s += masked(*reinterpret_cast<const uint32_t *>(gbase + d), d);
      d += 4;
    }
  }
  uint32_t le = fold(s);  // sum of little-endian words at even absolute offsets
  return (wa & 1) ? le : bswap16(le);
}

// An ICMP error message whose embedded IP header parsed.
__device__ __forceinline__ bool has_emb(const Hdr &H) { return H.emb != 0; }
// Sum (not complemented) of the ICMP checksum input of an error message with
// embedded headers: the ICMP header (checksum word excluded), then
// get_payload_for_checksum (icmp_any/checksum.rs:226-259) -- the embedded IP
// header, the embedded transport header and the payload, WITHOUT the
// embedded extension headers (as the reference computes it) -- and for
// ICMPv6 the pseudo header over that length (Icmpv6Type::calc_checksum).
__device__ __forceinline__ uint32_t icmp_err_sum(const Frame &F, const Hdr &H, const EmbV &E, int pay_start) {
  const int l = H.l4_off;
  uint64_t t = sum_frame(F, l, l + 2) + sum_frame(F, l + 4, l + H.l4_hlen);  // checksum word out
  t += sum_frame(F, E.off, E.off + E.net_hlen);
  t += sum_frame(F, E.t_off, E.t_off + E.t_len);
  t += sum_frame(F, pay_start, F.len);
  if (H.l4 == L4_ICMP6) {
    const uint32_t tl = (uint32_t)(H.l4_hlen + E.net_hlen + E.t_len + (F.len - pay_start));
    t += sum_frame(F, H.net_off + 8, H.net_off + 40);
    t += (tl >> 16) + (tl & 0xffff) + 58u;
  }
  return fold(t);
}
// IPv4 header checksum of the embedded header as it stands (checksum word out)
__device__ __forceinline__ uint16_t emb_ipv4_ck(const Frame &F, const EmbV &E) {
  const uint64_t t = sum_frame(F, E.off, E.off + 10) + sum_frame(F, E.off + 12, E.off + E.net_hlen);
  return (uint16_t)~fold(t);
}

// IcmpErrorHandler with an empty flow table (nat/src/icmp_handler/nf.rs:61-120):
// IcmpErrorPacket::new needs an embedded IP header and transport
// (net/src/packet/icmp_err.rs:37-53; else IcmpErrorIncomplete), then
// src_vpcd (Unroutable), valid ICMP and embedded IPv4 checksums
// (validate_checksums, :71-87; InvalidChecksum) and a flow key -- ports, or
// an ICMP query identifier (net/src/flows/flow_key.rs:635-660;
// IcmpErrorIncomplete).  No flow exists, so the packet goes on.
__device__ __forceinline__ uint8_t icmp_error_check(const Frame &F, const Hdr &H, const State &S) {
  if (!has_emb(H)) return DP_DONE_ICMP_ERROR_INCOMPLETE;
  const EmbV E = emb_view(F, H);
  if (E.tk == L4_NONE) return DP_DONE_ICMP_ERROR_INCOMPLETE;
  if (!S.src_vni) return DP_DONE_UNROUTABLE;
  if ((uint16_t)~icmp_err_sum(F, H, E, S.pay_start) != F.be16(H.l4_off + 2)) return DP_DONE_INVALID_CHECKSUM;
  if (E.net == 4 && emb_ipv4_ck(F, E) != F.be16(E.off + 10)) return DP_DONE_INVALID_CHECKSUM;
  if (E.tk == L4_ICMP4 || E.tk == L4_ICMP6) {
    // identifier: a query message (v4 echo / timestamp, v6 echo); a full
    // header only for the decoded types (code 0), a partial one with >= 6 bytes
    const uint8_t t = F.b(E.t_off), c = F.b(E.t_off + 1);
    const bool q = E.tk == L4_ICMP6 ? (t == 128 || t == 129) : (t == 0 || t == 8 || t == 13 || t == 14);
    const bool id = E.full ? (q && c == 0) : (q && E.t_len >= 6);
    if (!id) return DP_DONE_ICMP_ERROR_INCOMPLETE;
  }
  return DONE_NONE;
}

// ---------------------------------------------------------------------------
// Flow table (the flows variant of the kernel only; dp_flow.h)
// ---------------------------------------------------------------------------
// The flow FlowLookup attached to the packet (PacketMeta.flow_info), as it
// stood when the burst started, and the flow-table effects the packet has;
// they are applied by the kernel after the per-packet body, wave-aggregated.
struct FlowPk {
  uint32_t slot;       // kNoSlot: none
  uint32_t state;      // its slot state word (the ref's tag)
  uint32_t related;    // the related flow's slot (kNoSlot: none) and its state when
  uint32_t related_tag;  // the pair was made: alive while that slot still holds it
  uint32_t dst_vni, fflags;
  int64_t genid;
  bool active;         // FlowStatus::Active
  uint32_t ev0, ev1;   // pair invalidations (the flow's slot): flow-filter, ACL deny (kNoSlot: none)
  uint32_t ev_mark;    // mark of ev1 (ACL deny at packet idx: idx + 1)
  bool sens;           // ACL allowed it as the reply of a flow-scope-allowed flow
  uint32_t def_acl, s_flags, s_oif, s_fib;
  uint32_t s_dvni, s_vrf, s_nh;  // dst_vni, vrf (bit 31: Some) and nh_ref at the ACL
  uint32_t ev2, ev2_tag; // an ICMP error's invalidation of the flow it found (kNoSlot: none)
  uint32_t pf_rec;       // its port-forwarding record (dpf::PfReq), kNoSlot: none
  bool deferred;         // reached PortForwarder in the first pass: finished by the replay
  uint32_t acl_rule6;    // the rule of an ACL verdict 6
};

__device__ __forceinline__ uint4 ld4(const void *p) { return *reinterpret_cast<const uint4 *>(p); }
__device__ __forceinline__ uint32_t le32_at(const Frame &F, int f) {
  return (uint32_t)F.b(f) | ((uint32_t)F.b(f + 1) << 8) | ((uint32_t)F.b(f + 2) << 16) |
         ((uint32_t)F.b(f + 3) << 24);
}
__device__ __forceinline__ uint32_t be16_bytes(const Frame &F, int f) {
  return ((uint32_t)F.b(f) << 8) | F.b(f + 1);
}

// FlowTable::lookup (flow-entry/src/flow_table/table.rs:267-275): linear
// probing from the key's hash; one 128-byte line per slot, whose state, key
// and FlowInfo words (the first 80 bytes) are fetched in one round trip.
// v / w: the found slot's words 48..63 (status, flags, dst_vni, related) and
// 64..79 (related_tag, mark, genid).
__device__ __forceinline__ uint32_t flow_probe(const dpf::FlowCtx &fc, const dpf::FKey &k, uint32_t &state,
                                               uint4 &v, uint4 &w) {
  uint32_t i = dpf::fkey_hash(k) & fc.mask;
  const uint32_t bound = fc.tmeta[0];  // moved by the bursts' own inserts (dp_nat_resolve)
#pragma unroll 1
  for (uint32_t p = 0; p <= bound; p++) {
    const dpf::FlowSlot *s = fc.slots + i;
    const uint4 a = ld4(&s->state), b = ld4(&s->src[0]), c = ld4(&s->dst[0]);
    v = ld4(&s->status);
    w = ld4(&s->related_tag);
    const uint32_t st = a.x & 3u;
    if (st == dpf::FS_EMPTY) return dpf::kNoSlot;
    if (st == dpf::FS_FULL && a.y == k.w[0] && a.z == k.w[1] && a.w == k.w[2] && b.x == k.w[3] &&
        b.y == k.w[4] && b.z == k.w[5] && b.w == k.w[6] && c.x == k.w[7] && c.y == k.w[8] &&
        c.z == k.w[9] && c.w == k.w[10]) {
      state = a.x;
      return i;
    }
    i = (i + 1) & fc.mask;
  }
  return dpf::kNoSlot;
}

// FlowKey::try_from(&Packet) (net/src/flows/flow_key.rs:589-621).  false: no
// key, or an ICMP error message's key (IcmpProtoKey::ErrorMsgData), which no
// stored flow has.
__device__ __forceinline__ bool packet_fkey(const Frame &F, const Hdr &H, const State &S, dpf::FKey &k) {
  if (H.net == 0) return false;
  uint32_t kind, ports = 0;
  if (H.l4 == L4_TCP || H.l4 == L4_UDP) {
    kind = H.l4 == L4_TCP ? DP_FLOW_TCP : DP_FLOW_UDP;
    ports = ((uint32_t)S.sport << 16) | S.dport;
  } else if (H.l4 == L4_ICMP4 || H.l4 == L4_ICMP6) {
    // IcmpProtoKey::new_icmp_v4/v6 (flow_key.rs:318-338): Echo Request / Reply
    const bool v6 = H.l4 == L4_ICMP6;
    const uint8_t t = F.b(H.l4_off), c = F.b(H.l4_off + 1);
    if (c == 0 && (v6 ? (t == 128 || t == 129) : (t == 0 || t == 8))) {
      kind = DP_FLOW_ICMP_QUERY;
      ports = be16_bytes(F, H.l4_off + 4) << 16;
    } else if (icmp_err_at(F, H.l4_off, v6)) {
      return false;
    } else {
      kind = DP_FLOW_ICMP_OTHER;
    }
  } else {
    return false;
  }
  k.w[0] = S.src_vni;
  k.w[1] = (H.net == 4 ? 4u : 6u) | (kind << 8);
  k.w[2] = ports;
  // the address words as plain values per branch, then stored once: the key
  // written field by field in either branch was kept in scratch memory (a
  // store and a reload ahead of the flow hash)
  uint32_t a[8];
  if (H.net == 4) {
    a[0] = __builtin_bswap32(S.v4src);
    a[4] = __builtin_bswap32(S.v4dst);
    a[1] = a[2] = a[3] = a[5] = a[6] = a[7] = 0;
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      a[j] = le32_at(F, H.net_off + 8 + 4 * j);
      a[4 + j] = le32_at(F, H.net_off + 24 + 4 * j);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; j++) k.w[3 + j] = a[j];
  return true;
}

// Attach a found flow (PacketMeta.flow_info): its FlowInfo as the burst started.
__device__ __forceinline__ void flow_attach(uint32_t slot, uint32_t state, const uint4 &v, const uint4 &w,
                                            FlowPk &fp) {
  fp.slot = slot;
  fp.state = state;
  fp.active = v.x == DP_FLOW_ACTIVE;
  fp.fflags = v.y;
  fp.dst_vni = v.z;
  fp.related = v.w;
  fp.related_tag = w.x;
  fp.genid = (int64_t)(((uint64_t)w.w << 32) | w.z);
}

// handle_icmp_error_masquerading (nat/src/masquerade/icmp_handling.rs:16-48)
// for the active flow an overlay ICMP error names: the embedded packet by the
// state's reverse_translation_data (state.rs:89-98: a SrcNat state restores
// the inner destination, a DstNat state the inner source, with its TCP / UDP
// port or -- translate_inner_icmp, icmp_error_msg.rs:149-173 -- its ICMP
// identifier), then the error itself by the state (masquerade, packet.rs:
// 35-195: the address; an error message carries no identifier).  Any failure
// is InternalFailure.  An unrecoverable error on a one-way flow invalidates
// the pair (before any flow-filter decision of the burst: mark 0).
__device__ __forceinline__ void icmp_error_masq(const dpf::FlowCtx &fc, const Frame &F, const Hdr &H, State &S,
                                             FlowPk &fp, uint32_t sl, uint32_t st) {
  const EmbV E = emb_view(F, H);
  const dpf::FlowSlot *fs = fc.slots + sl;
  const uint4 pfa = ld4(&fs->pf), pfb = ld4(&fs->pf_ip[2]);
  const uint32_t act = pfa.x & 0xffu, nfs = (pfa.x >> 8) & 0xffu, port = pfa.x >> 16;
  const uint32_t ip[4] = {pfa.z, pfa.w, pfb.x, pfb.y};
  const uint32_t fam = pfb.z;
  const bool inner_src = act == DP_PF_DST_NAT;
  const bool unicast = fam == 4 ? !((ip[0] >> 28) == 0xe || ip[0] == 0xffffffffu) : (ip[0] >> 24) != 0xff;
  // the inner side needs a unicast address (DstNat), the outer one too (SrcNat)
  if ((int)fam != E.net || !unicast) { done(S, DP_DONE_INTERNAL_FAILURE); return; }
  const int ao = E.off + (E.net == 4 ? (inner_src ? 12 : 16) : (inner_src ? 8 : 24));
  for (int j = 0; j < (E.net == 4 ? 1 : 4); j++) wput32(F, ao + 4 * j, ip[j]);
  if (E.tk == L4_TCP || E.tk == L4_UDP) {
    if (port == 0) { done(S, DP_DONE_INTERNAL_FAILURE); return; }  // InvalidPort
    if (F.be16(E.t_off + (inner_src ? 0 : 2)) != port) wput16(F, E.t_off + (inner_src ? 0 : 2), port);
  } else if (inner_src && F.be16(E.t_off + 4) != port) {
    // the embedded ICMP query's identifier (icmp_error_check: it has one)
    wput16(F, E.t_off + 4, port);
  }
  const bool osrc = act == DP_PF_SRC_NAT;
  bool mod = false;
  if (H.net == 4) {
    uint32_t &a = osrc ? S.v4src : S.v4dst;
    if (a != ip[0]) { a = ip[0]; mod = true; }
  } else {
    const int oo = H.net_off + (osrc ? 8 : 24);
    for (int j = 0; j < 4; j++)
      if (F.be32(oo + 4 * j) != ip[j]) { wput32(F, oo + 4 * j, ip[j]); mod = true; }
  }
  if (mod) S.flags |= DP_META_REFR_CHKSUM | (osrc ? DP_META_NATTED_SRC : DP_META_NATTED_DST);
  const uint8_t t = F.b(H.l4_off), c = F.b(H.l4_off + 1);
  const bool unrec = H.l4 == L4_ICMP4 ? (t == 3 && c != 4) : t == 1;
  if (unrec && nfs == DP_NFS_ONE_WAY) { fp.ev2 = sl; fp.ev2_tag = st; }
  S.flags |= DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST;
}

// IcmpErrorHandler with a flow table (nat/src/icmp_handler/nf.rs:102-152):
// the embedded packet's flow key, reversed, from the error's source VPC
// (embedded_flowkey flow_key.rs:635-660, FlowKey::reverse :567-576).  A flow
// found inactive filters the error; an active one sets the destination VPC
// and -- with no masquerade / port-forwarding state to translate with --
// filters it too.  Runs after icmp_error_check accepted the message.
__device__ __forceinline__ void icmp_error_flow(const dpf::FlowCtx &fc, const Frame &F, const Hdr &H, State &S,
                                                FlowPk &fp) {
  const EmbV E = emb_view(F, H);
  dpf::FKey k;
  uint32_t kind, ports;
  if (E.tk == L4_TCP || E.tk == L4_UDP) {
    kind = E.tk == L4_TCP ? DP_FLOW_TCP : DP_FLOW_UDP;
    ports = (be16_bytes(F, E.t_off + 2) << 16) | be16_bytes(F, E.t_off);
  } else {
    kind = DP_FLOW_ICMP_QUERY;
    ports = be16_bytes(F, E.t_off + 4) << 16;
  }
  k.w[0] = S.src_vni;
  k.w[1] = (uint32_t)E.net | (kind << 8);
  k.w[2] = ports;
  const int so = E.net == 4 ? 12 : 8, dof = E.net == 4 ? 16 : 24;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const bool w = E.net == 6 || j == 0;
    k.w[3 + j] = w ? le32_at(F, E.off + dof + 4 * j) : 0u;
    k.w[7 + j] = w ? le32_at(F, E.off + so + 4 * j) : 0u;
  }
  uint32_t st;
  uint4 v, w;
  const uint32_t sl = flow_probe(fc, k, st, v, w);
  if (sl == dpf::kNoSlot) return;  // no flow: let it through (nf.rs:114-121)
  if (v.x != DP_FLOW_ACTIVE) { done(S, DP_DONE_FILTERED); return; }  // nf.rs:126-130
  S.dst_vni = v.z;                                                   // nf.rs:139-140
  if (!SNAT || !(v.y & (dpf::kFlagPf | dpf::kFlagMasq))) { done(S, DP_DONE_FILTERED); return; }  // no NAT state (:143-152)
#ifdef DP_X_NOICMP
  return;
#endif
  if (v.y & dpf::kFlagMasq) { icmp_error_masq(fc, F, H, S, fp, sl, st); return; }
  // handle_icmp_error_port_forwarding (nat/src/portfw/icmp_handling.rs:51-90):
  // the embedded packet back to its form before the flow's translation
  // (nat_translate_icmp_inner, icmp_error_msg.rs:46-146: DstNat state ->
  // the inner source, SrcNat -> the inner destination, address and TCP / UDP
  // port), then the error itself NATed by the state (nat_packet: its address)
  const dpf::FlowSlot *fs = fc.slots + sl;
  const uint4 pfa = ld4(&fs->pf), pfb = ld4(&fs->pf_ip[2]);
  const uint32_t act = pfa.x & 0xffu, nfs = (pfa.x >> 8) & 0xffu, port = pfa.x >> 16;
  const uint32_t ip[4] = {pfa.z, pfa.w, pfb.x, pfb.y};
  const uint32_t fam = pfb.z;
  const bool inner_src = act == DP_PF_DST_NAT;
  const bool unicast = fam == 4 ? !((ip[0] >> 28) == 0xe || ip[0] == 0xffffffffu) : (ip[0] >> 24) != 0xff;
  if ((int)fam != E.net || (inner_src && !unicast)) { done(S, DP_DONE_INTERNAL_FAILURE); return; }
  const int ao = E.off + (E.net == 4 ? (inner_src ? 12 : 16) : (inner_src ? 8 : 24));
  for (int j = 0; j < (E.net == 4 ? 1 : 4); j++) wput32(F, ao + 4 * j, ip[j]);
  if ((E.tk == L4_TCP || E.tk == L4_UDP) && F.be16(E.t_off + (inner_src ? 0 : 2)) != port)
    wput16(F, E.t_off + (inner_src ? 0 : 2), port);
  // the outer header: an ICMP message keeps its ports, only the address moves
  const bool osrc = act == DP_PF_SRC_NAT;
  bool mod = false;
  if (H.net == 4) {
    uint32_t &a = osrc ? S.v4src : S.v4dst;
    if (a != ip[0]) { a = ip[0]; mod = true; }
  } else {
    const int oo = H.net_off + (osrc ? 8 : 24);
    for (int j = 0; j < 4; j++)
      if (F.be32(oo + 4 * j) != ip[j]) { wput32(F, oo + 4 * j, ip[j]); mod = true; }
  }
  if (mod) S.flags |= DP_META_REFR_CHKSUM | (osrc ? DP_META_NATTED_SRC : DP_META_NATTED_DST);
  // is_icmp_unrecoverable (nf.rs:42-60) with a one-way flow: the pair goes
  // (before any flow-filter decision of the burst: mark 0)
  const uint8_t t = F.b(H.l4_off), c = F.b(H.l4_off + 1);
  const bool unrec = H.l4 == L4_ICMP4 ? (t == 3 && c != 4) : t == 1;
  if (unrec && nfs == DP_NFS_ONE_WAY) { fp.ev2 = sl; fp.ev2_tag = st; }
  S.flags |= DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST;  // nf.rs:176-179
}

// ---------------------------------------------------------------------------
// Stages
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool find_iface(const Img &g, uint32_t ifx, IfRec &out) {
  if (ifx < g.im.if_direct_n) {
    out = g.at<IfRec>(g.im.if_direct)[ifx];
    return out.valid != 0;
  }
  uint32_t idx;
  if (!hash_find(g, g.im.ifaces, ifx, 0, 0, idx)) return false;
  out = g.at<IfRec>(g.im.if_recs)[idx];
  return true;
}

__device__ __forceinline__ void stage_ingress(const Img &g, const Frame &F, const Hdr &H, State &S, uint32_t iif) {
  if (S.done != DONE_NONE) return;
  IfRec I;
  if (!find_iface(g, iif, I)) { done(S, DP_DONE_INTERFACE_UNKNOWN); return; }
  if (I.pre_code != 255) { done(S, I.pre_code); return; }
  if (S.edst == 0xffffffffffffull) { S.flags |= DP_META_IS_L2_BCAST; done(S, DP_DONE_UNHANDLED); return; }
  if (S.edst != I.mac) { done(S, DP_DONE_MAC_NOT_FOR_US); return; }
  if (I.post_code != 255) { done(S, I.post_code); return; }
  if (H.net == 0) { done(S, DP_DONE_NOT_IP); return; }
  S.has_vrf = true;
  S.vrf = I.vrf_id;
  S.fib = I.fib;
}

// VNI -> VniRec (the VNI's FIB, VRF and per-VNI tables)
// VNI map probe: the slots are the VniRecs themselves (vni 0 = empty)
__device__ __forceinline__ int32_t find_vni(const Img &g, uint32_t vni) {
  if (vni == 0) return -1;
  const CTX_AS VniRec *slots = CTX_TAB(VniRec, 0, g.im.vni_slots);
  const uint32_t mask = g.im.vni_mask;
  uint32_t i = hmix(vni, 0, 0) & mask;
  for (uint32_t probe = 0; probe <= mask; probe++) {
    TRIP();
    const uint32_t k = slots[i].vni;
    if (k == vni) return (int32_t)i;
    if (k == 0) return -1;
    i = (i + 1) & mask;
  }
  return -1;
}

__device__ __forceinline__ bool enter_vni(const Img &g, State &S, uint32_t vni) {
  const int32_t vi = find_vni(g, vni);
  if (vi < 0) return false;
  const auto &R = VNI_REC(vi);
  S.src_vni = vni;
  S.has_vrf = true;
  S.vrf = R.vrf_id;
  S.fib = (int32_t)R.fib;
  S.vni_idx = (int32_t)vi;
  S.flags |= DP_META_IS_OVERLAY;
  return true;
}

// PairRec of (src_vni, dst_vni): from the flow-filter verdict, else by lookup
__device__ __forceinline__ int32_t pair_of(const Img &g, State &S) {
  if (S.pair < 0) {
    uint32_t pi;
    if (pair_find(g, S.src_vni, S.dst_vni, pi)) S.pair = (int32_t)pi;
  }
  return S.pair;
}

__device__ __forceinline__ void decrement_ttl(State &S) {
  if (S.ttl == 0) { done(S, DP_DONE_HOP_LIMIT_EXCEEDED); return; }
  S.ttl--;
  if (S.ttl == 0) done(S, DP_DONE_HOP_LIMIT_EXCEEDED);
}

// IPv4 header checksum of the current inner header (with current fields)
__device__ __forceinline__ uint16_t ipv4_csum(const Frame &F, const Hdr &H, const State &S) {
  int o = H.net_off;
  uint64_t s = 0;
  s += ((uint32_t)F.b(o) << 8) | F.b(o + 1);
  s += F.be16(o + 2);
  s += F.be16(o + 4);
  s += ((uint32_t)(F.b(o + 6) & 0x7f) << 8) | F.b(o + 7);  // reserved bit not kept
  s += ((uint32_t)S.ttl << 8) | F.b(o + 9);
  s += (S.v4src >> 16) + (S.v4src & 0xffff) + (S.v4dst >> 16) + (S.v4dst & 0xffff);
  for (int i = 20; i < H.net_hlen; i += 2) s += F.be16(o + i);
  return (uint16_t)~fold(s);
}

// Full L4 checksum of the current (inner) headers over the payload
__device__ __forceinline__ uint16_t l4_csum(const Frame &F, const Hdr &H, const State &S) {
  int plen = F.len - S.pay_start;
  uint32_t pay = sum_frame(F, S.pay_start, F.len);
  uint64_t s = pay;
  if (H.l4 == L4_UDP) {
    uint16_t ulen = F.be16(H.l4_off + 4);
    if (H.net == 4) s += (S.v4src >> 16) + (S.v4src & 0xffff) + (S.v4dst >> 16) + (S.v4dst & 0xffff) + 17 + ulen;
    else { for (int i = 0; i < 32; i += 2) s += F.be16(H.net_off + 8 + i); s += ulen + 17; }
    s += S.sport + S.dport + ulen;
    uint16_t c = (uint16_t)~fold(s);
    return c == 0 ? 0xffff : c;
  }
  if (H.l4 == L4_TCP) {
    uint32_t tl = (uint32_t)H.l4_hlen + (uint32_t)plen;
    if (H.net == 4) s += (S.v4src >> 16) + (S.v4src & 0xffff) + (S.v4dst >> 16) + (S.v4dst & 0xffff) + 6 + (tl & 0xffff);
    else { for (int i = 0; i < 32; i += 2) s += F.be16(H.net_off + 8 + i); s += (tl >> 16) + (tl & 0xffff) + 6; }
    int o = H.l4_off;
    s += S.sport + S.dport;
    s += F.be16(o + 4) + F.be16(o + 6) + F.be16(o + 8) + F.be16(o + 10);
    s += ((uint32_t)(F.b(o + 12) & 0xf1) << 8) | F.b(o + 13);  // reserved bits not kept
    s += F.be16(o + 14) + F.be16(o + 18);
    for (int i = 20; i < H.l4_hlen; i += 2) s += F.be16(o + i);
    return (uint16_t)~fold(s);
  }
  if (H.l4 == L4_ICMP4 || H.l4 == L4_ICMP6) {
    int o = H.l4_off;
    s += F.be16(o);
    for (int i = 4; i < H.l4_hlen; i += 2) s += F.be16(o + i);
    if (H.l4 == L4_ICMP6) {
      uint32_t tl = (uint32_t)H.l4_hlen + (uint32_t)plen;
      for (int i = 0; i < 32; i += 2) s += F.be16(H.net_off + 8 + i);
      s += (tl >> 16) + (tl & 0xffff) + 58;
    }
    return (uint16_t)~fold(s);
  }
  return 0;
}

__device__ __forceinline__ void vxlan_encap(const Img &g, const Frame &F, const Hdr &H, State &S, const Instr &in, const FibRec &fb) {
  if (!(fb.flags & DP_FIB_VTEP_HAS_MAC)) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  if (!(in.flags & DP_INSTR_HAS_DMAC)) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  uint8_t vz = 0, dz = 0;
  for (int i = 0; i < 6; i++) { vz |= fb.vtep_mac[i]; dz |= in.mac[i]; }
  if (vz == 0 || (fb.vtep_mac[0] & 1)) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  S.esrc = load_mac(fb.vtep_mac);
  if (dz == 0) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); S.eth_dirty = true; return; }
  S.edst = load_mac(in.mac);
  S.eth_dirty = true;
  // inner checksums (IpForwarder::vxlan_encap): the IPv4 header checksum
  // always, the full L4 checksum if REFR_CHKSUM; computed at serialize from
  // the same (then unchanged) inner fields
  if (S.flags & DP_META_REFR_CHKSUM) {
    S.inner_l4_ck = (H.l4 != L4_NONE) && !H.vx;
    S.flags &= ~DP_META_REFR_CHKSUM;
  } else if (H.net == 4) {
    S.inner_l4_ck = false;
  } else {
    done(S, DP_DONE_INTERNAL_FAILURE);  // unreachable!() in the reference
    return;
  }
  if (!(fb.flags & DP_FIB_VTEP_HAS_IP)) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  if (fb.vtep_fam == 4 && in.fam == 4) {
    uint32_t s4 = ((uint32_t)fb.vtep_ip[0] << 24) | ((uint32_t)fb.vtep_ip[1] << 16) | ((uint32_t)fb.vtep_ip[2] << 8) | fb.vtep_ip[3];
    if ((s4 >> 28) == 0xe || s4 == 0xffffffffu) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); return; }
    S.o_fam = 4;
  } else if (fb.vtep_fam == 6 && in.fam == 6) {
    if (fb.vtep_ip[0] == 0xff) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); return; }
    S.o_fam = 6;
  } else {
    done(S, DP_DONE_VXLAN_ENCAP_FAILURE);
    return;
  }
  OuterHdr ob;
  for (int i = 0; i < 4; i++) {
    ob.src.w[i] = ((uint32_t)fb.vtep_ip[4 * i] << 24) | ((uint32_t)fb.vtep_ip[4 * i + 1] << 16) | ((uint32_t)fb.vtep_ip[4 * i + 2] << 8) | fb.vtep_ip[4 * i + 3];
    ob.dst.w[i] = ((uint32_t)in.addr[4 * i] << 24) | ((uint32_t)in.addr[4 * i + 1] << 16) | ((uint32_t)in.addr[4 * i + 2] << 8) | in.addr[4 * i + 3];
  }
  if (S.o_fam == 4) { ob.src.w[1] = ob.src.w[2] = ob.src.w[3] = 0; ob.dst.w[1] = ob.dst.w[2] = ob.dst.w[3] = 0; }
  // headroom check of the prepend (Packet::vxlan_encap): inner headers go
  // right before the payload; we only fail if they would not fit at all.
  int inner_start = S.pay_start - H.size;
  if (inner_start < -(int)DP_HEADROOM) { done(S, DP_DONE_VXLAN_ENCAP_FAILURE); return; }
  // packet_hash_vxlan over the (updated) inner headers
  HBuf hbuf{F.hs, 0};
  hb_usize(hbuf, 6);  // source(): a [u8; 6] hashes as a slice -- length prefix, then the bytes
  for (int i = 0; i < 6; i++) hb_put(hbuf, mac_b(S.esrc, i));
  hb_usize(hbuf, 6);  // destination()
  for (int i = 0; i < 6; i++) hb_put(hbuf, mac_b(S.edst, i));
  hb_u16(hbuf, ((uint32_t)F.b(H.hb + 12) << 8) | F.b(H.hb + 13));  // ether_type(): write_u16
  for (int v = 0; v < H.nvlan; v++) hb_u16(hbuf, F.be16(H.hb + 14 + 4 * v) & 0x0fff);  // vid(): write_u16
  hash_ip_fields(F, H, S, hbuf);
  uint64_t x = rapid(hbuf.b, hbuf.n);
  ob.sport = (uint16_t)(x % 16384 + 49152);
  ob.len = (uint16_t)((F.len - S.pay_start) + H.size + 16);
  ob.tos = S.has_dscp ? (uint8_t)((S.dscp << 2) | S.ecn) : 0;
  ob.vni = in.vni;
  ob.fam = S.o_fam;
  // deparse the outer IP/UDP/VXLAN now, over the dead hash input: none of it
  // stays live in registers until serialize (Egress adds the outer Ethernet)
  lds_u8 *o = F.hs;
  int u;  // UDP header offset
  if (ob.fam == 4) {
    hput16(o, 0, 0x4500u | ob.tos);
    hput16(o, 2, 20u + ob.len);
    hput16(o, 4, 0);
    hput16(o, 6, 0x4000u);                 // Ipv4Header::default(): DF
    hput16(o, 8, (64u << 8) | 17u);
    hput16(o, 10, outer_ck4(ob));
    hput32(o, 12, ob.src.w[0]);
    hput32(o, 16, ob.dst.w[0]);
    u = 20;
  } else {
    hput32(o, 0, (0x60000000u | ((uint32_t)ob.tos << 20)));
    hput16(o, 4, ob.len);
    hput16(o, 6, (17u << 8) | 64u);
#pragma unroll
    for (int k = 0; k < 4; k++) { hput32(o, 8 + 4 * k, ob.src.w[k]); hput32(o, 24 + 4 * k, ob.dst.w[k]); }
    u = 40;
  }
  hput16(o, u, ob.sport);
  hput16(o, u + 2, 4789u);
  hput16(o, u + 4, ob.len);
  hput16(o, u + 6, 0);                     // outer UDP checksum 0
  hput32(o, u + 8, 0x08000000u);           // VXLAN flags: I
  hput32(o, u + 12, ob.vni << 8);
  S.encap = true;
  S.dst_vni = in.vni;
}

__device__ __forceinline__ void stage_ipforward(const Img &g, const Frame &F, Hdr &H, State &S) {
  if (S.done != DONE_NONE) return;
  bool had_vrf = S.has_vrf;
  uint32_t vrf0 = S.vrf;
  int32_t fi;
  uint64_t d4 = 0, k4 = 0;   // the dst FIB's v4 LPM, read from the pair context (no FibRec load)
  uint32_t b4 = 0;
  if (S.dst_vni) {
    if (H.net == 0 && !S.encap) { done(S, DP_DONE_INTERNAL_FAILURE); return; }
    int32_t pi = pair_of(g, S);
    if (pi >= 0) {
      const auto &PR = PAIR_REC(pi);
      fi = PR.dst_fib;
      d4 = PR.lpm4_direct;
      b4 = PR.lpm4_dbits;
      k4 = PR.lpm4_blocks;
    } else {
      const int32_t vi = find_vni(g, S.dst_vni);
      fi = vi >= 0 ? (int32_t)CTX_TAB(VniRec, 0, g.im.vni_slots)[vi].fib : -1;
    }
    if (fi < 0) { done(S, DP_DONE_INTERNAL_FAILURE); return; }
  } else if (S.has_vrf) {
    if (H.net == 0) { done(S, DP_DONE_INTERNAL_FAILURE); return; }
    fi = S.fib;
    if (fi < 0) { done(S, DP_DONE_INTERNAL_FAILURE); return; }
  } else {
    if (S.flags & DP_META_IS_OVERLAY) done(S, DP_DONE_INTERNAL_FAILURE);
    return;
  }
  if (S.encap) { done(S, DP_DONE_INTERNAL_FAILURE); return; }  // routing an encapsulated packet again: unsupported
  const FibRec &fb = g.at<FibRec>(g.im.fibs)[fi];  // fields read where used (no struct copy)
  uint8_t fam; uint64_t khi, klo;
  cur_dst_key(F, H, S, fam, khi, klo);
  // one walk for every lane: v4 and v6 lanes of a wave issue their direct-table
  // loads together (two call sites would run one after the other)
  uint32_t sel = 0;
  if (!(fam == 4 && d4)) {
    const Lpm &L = fam == 4 ? fb.v4 : fb.v6;
    d4 = L.direct;
    b4 = L.dbits;
    k4 = L.blocks;
    // a v6 key inside the FIB's window reads the window table instead
    if (DP_V6W && fam == 6 && L.wtab && (khi >> (64 - L.wbits)) == L.wpfx) {
      d4 = L.wtab;
      k4 = 0;
      sel = lpm_sel(L.wbits + L.wtb, 64 - L.wbits - L.wtb, L.wtb);
    }
  }
  if (!sel) sel = lpm_dsel(b4);
  const uint32_t nhi = lpm_walk(g, d4, sel, k4, khi, klo);
  TRIP();
  const auto &nr = CTX_REC(NhRec, g.im.ctx_nh, g.im.nh_recs, nhi);
  if (nr.kind != DPD_NH_CHAIN) {
    // a single Egress / Drop instruction, resolved at publish (NhRec)
    S.fib_entry = nr.entry;
    decrement_ttl(S);
    if (S.done != DONE_NONE) return;
    if (nr.kind == DPD_NH_DROP) { done(S, DP_DONE_ROUTE_DROP); return; }
    S.nh_ref = NH_ENTRY | nr.entry;  // the entry's one Egress instruction
    S.has_oif = nr.has_oif;
    S.oif = nr.oif;
    S.eg_code = nr.eg_code;
    S.if_code = nr.if_code;
    S.eg_dmac = nr.eg_dmac;
    S.eg_smac = nr.eg_smac;
    if (S.has_vrf == had_vrf && (!had_vrf || S.vrf == vrf0)) S.has_vrf = false;
    return;
  }
  uint32_t idx = 0;
  if (nr.n_entries > 1) {
    HBuf hbuf{F.hs, 0};
    hash_ip_fields(F, H, S, hbuf);
    idx = (uint32_t)(rapid(hbuf.b, hbuf.n) % nr.n_entries);
  }
  uint32_t ei = nr.entry + idx;
  TRIP();
  const Entry E = g.at<Entry>(g.im.entries)[ei];
  S.fib_entry = ei;
  const Instr *ins = g.at<Instr>(g.im.instrs) + E.first_instr;
  bool iplocal = E.n_instr == 1 && ins[0].kind == DP_INSTR_LOCAL;
  if (!iplocal) {
    decrement_ttl(S);
    if (S.done != DONE_NONE) return;
  }
  for (uint32_t k = 0; k < E.n_instr; k++) {
    const Instr &in = ins[k];
    switch (in.kind) {
      case DP_INSTR_DROP: done(S, DP_DONE_ROUTE_DROP); break;
      case DP_INSTR_LOCAL: {
        if (!H.vx) { done(S, DP_DONE_LOCAL); break; }
        uint8_t tos = 0;
        bool has_q = H.net != 0;
        if (H.net == 4) tos = F.b(H.net_off + 1);
        if (H.net == 6) tos = (uint8_t)(((F.b(H.net_off) & 0xf) << 4) | (F.b(H.net_off + 1) >> 4));
        uint32_t vni = H.vni;
        Hdr I;
        if (!parse(F, H.hb + H.consumed, I)) { done(S, DP_DONE_VXLAN_DECAP_FAILURE); break; }
        H = I;
        load_fields(F, H, S);
        if (has_q) { S.has_dscp = true; S.dscp = tos >> 2; S.ecn = tos & 3; }
        if (!enter_vni(g, S, vni)) { done(S, DP_DONE_UNROUTABLE); break; }
        break;
      }
      case DP_INSTR_ENCAP_VXLAN: vxlan_encap(g, F, H, S, in, fb); break;
      case DP_INSTR_EGRESS:
        S.nh_ref = E.first_instr + k;
        S.has_oif = in.flags & DP_INSTR_HAS_IFINDEX;
        S.oif = in.ifindex;
        S.eg_code = in.eg_code;
        S.if_code = in.if_code;
        S.eg_dmac = in.eg_dmac;
        S.eg_smac = in.eg_smac;
        break;
    }
    if (S.done != DONE_NONE) return;
  }
  if (S.has_vrf == had_vrf && (!had_vrf || S.vrf == vrf0)) S.has_vrf = false;
}

__device__ __forceinline__ Key128 key_of(const Frame &F, const Hdr &H, const State &S, bool src) {
  if (H.net == 4) return Key128{0, src ? S.v4src : S.v4dst};
  int o = H.net_off + (src ? 8 : 24);
  Key128 k;
  k.hi = ((uint64_t)F.be32(o) << 32) | F.be32(o + 4);
  k.lo = ((uint64_t)F.be32(o + 8) << 32) | F.be32(o + 12);
  return k;
}

// Hoisted index walks.  After the flow-filter remote verdict the next stages
// -- flow-filter local, ACL, static NAT src and dst -- each start with a
// multibit index walk that depends only on the VNI pair and the packet's
// fields.  They run here in lockstep so their dependent loads overlap; the
// stages continue from the leaves (NO_PRE: not hoisted -- v6, an absent
// table, a bit-vector group or a bounds-form index; the stage walks itself).
struct Pre { uint32_t ffl, acl, nsrc, ndst; };

// The shorter of two candidate runs of one ACL group (the run of the packet's
// interval in the group's first and second list index): either holds every
// rule that can match, in precedence order.
__device__ __forceinline__ uint32_t shorter_run(uint32_t a, uint32_t b) {
  if (b == NO_PRE) return a;
  return (b & DPD_RUN_MAX) < (a & DPD_RUN_MAX) ? b : a;
}

// Key of a classifier field for the v4 hoisted walks (f: 0 src, 1 dst, 2
// sport, 3 dport); `local` = the flow-filter local table, whose dst / dport
// keys are wildcards (0).
__device__ __forceinline__ uint32_t mbi_key(const State &S, uint32_t f, bool local) {
  return f == 0 ? S.v4src : f == 1 ? (local ? 0u : S.v4dst) : f == 2 ? (uint32_t)S.sport
                                                                     : (local ? 0u : (uint32_t)S.dport);
}

__device__ __forceinline__ void hoist_walks(const Img &g, const State &S, int32_t pi, Pre &P) {
  P.ffl = P.acl = P.nsrc = P.ndst = NO_PRE;
  // the index descriptors ride in the pair / VNI contexts (Mbi): the four
  // walks start right after the pair context arrives
  const auto &PR = PAIR_REC(pi);
  const auto &VR = VNI_REC(S.vni_idx);
#ifndef DP_TWO_ACL_INDEX
  constexpr int NW = 4;
  Mbi m[NW] = {PR.ffl4, PR.acl4, PR.nsrc, VR.ndst};
#else
  // experiment (negative results): a fifth walk over the ACL
  // group's second list index, verifying the shorter run
  constexpr int NW = 5;
  Mbi m[NW] = {PR.ffl4, PR.acl4, PR.nsrc, VR.ndst, PR.acl4b};
#endif
  uint32_t key[NW], e[NW];
  int rem0[NW];
  key[0] = mbi_key(S, m[0].field, true);
  key[1] = mbi_key(S, m[1].field, false);
  key[2] = S.v4src;
  key[3] = S.v4dst;
  if constexpr (NW > 4) key[NW - 1] = mbi_key(S, m[NW - 1].field, false);
#pragma unroll
  for (int k = 0; k < NW; k++) {
    rem0[k] = (int)m[k].kbits - (int)m[k].s0;
    e[k] = m[k].root ? g.at<uint32_t>(m[k].root)[key[k] >> rem0[k]] : DPD_LEAF;
  }
  TRIP();
#pragma unroll
  for (int l = 1; l <= 3; l++) {
    uint32_t all = DPD_LEAF;
#pragma unroll
    for (int k = 0; k < NW; k++) all &= e[k];
    if (!all) TRIP();
#pragma unroll
    for (int k = 0; k < NW; k++)
      if (!(e[k] & DPD_LEAF)) e[k] = g.at<uint32_t>(m[k].blocks)[(e[k] << 8) | ((key[k] >> (rem0[k] - 8 * l)) & 0xff)];
  }
  if (m[0].root) P.ffl = e[0] & ~DPD_LEAF;
  if (m[1].root) P.acl = shorter_run(e[1] & ~DPD_LEAF, (NW > 4 && m[NW - 1].root) ? e[NW - 1] & ~DPD_LEAF : NO_PRE);
  if (m[2].root) P.nsrc = e[2] & ~DPD_LEAF;
  if (m[3].root) P.ndst = e[3] & ~DPD_LEAF;
}

// FlowFilter (flow-filter/src/lib.rs:75-246).  FL: with a flow table -- an
// attached flow that is active and not outdated bypasses the tables
// (dst_vpcd_from_valid_flow / tag_for_bypass, lib.rs:122-131,213-231,327-349);
// a miss invalidates the attached flow pair, and so does a hit for a flow of
// another generation (should_invalidate_flow, :258-294: without masquerade /
// port-forwarding state an outdated flow is either misrouted or no longer
// needed).  Flows carry no such state, so revalidation (flow_revalidation_data,
// :296-325) is the plain lookup.
template <bool FL>
__device__ __forceinline__ void stage_flow_filter(const Img &g, const Frame &F, const Hdr &H, State &S, Pre &P,
                                                  FlowPk &fp, const dpf::FlowCtx *fc, const dpf::PfReq *rp) {
  P.ffl = P.acl = P.nsrc = P.ndst = NO_PRE;
  if (S.done != DONE_NONE || !(S.flags & DP_META_IS_OVERLAY) || S.dst_vni) return;
  uint8_t gate = 0;  // SourceGate of the local lookup
  uint32_t gate_vni = 0;  // GateVni of the remote lookup (LookupInput.dst_vpcd; 0: None)
  // FL: a bypassing lane (its flow decides) skips the tables, but joins the
  // other lanes where they start the ACL's and static NAT's hoisted index
  // walks, so its walks go out with theirs instead of one after the other
  // in those stages
  bool byp = false;
  if constexpr (FL) {
    if (rp) {
      // the replay: the first pass's verdict from the record (its
      // destination VPC and requirements), no classifier walk
      S.dst_vni = rp->dst_vni;
      if (rp->bits & dpf::kPqSnatSrc) S.flags |= DP_META_REQ_STATIC_NAT_SRC;
      if (rp->bits & dpf::kPqSnatDst) S.flags |= DP_META_REQ_STATIC_NAT_DST;
      if (SNAT && (rp->bits & dpf::kPqPf)) S.flags |= DP_META_REQ_PORT_FORWARDING;
      if (SNAT && (rp->bits & dpf::kPqMasq)) S.flags |= DP_META_REQ_MASQUERADE;
      return;
    }
    if (fp.slot != dpf::kNoSlot && fp.active && fp.genid >= fc->genid) {
      S.dst_vni = fp.dst_vni;
      if (SNAT && (fp.fflags & dpf::kFlagMasq)) S.flags |= DP_META_REQ_MASQUERADE;
      if (SNAT && (fp.fflags & dpf::kFlagPf)) S.flags |= DP_META_REQ_PORT_FORWARDING;
      if (fp.fflags & DP_FLOW_REQ_STATIC_NAT_SRC) S.flags |= DP_META_REQ_STATIC_NAT_SRC;
      if (fp.fflags & DP_FLOW_REQ_STATIC_NAT_DST) S.flags |= DP_META_REQ_STATIC_NAT_DST;
      byp = true;
    }
    // flow_revalidation_data (:296-325): the reply flow of a masqueraded pair
    // is revalidated against the remote rules gated on its destination VPC,
    // that of a port-forwarded pair against the local rules gated on
    // PortFwdReply
    else if (SNAT && fp.slot != dpf::kNoSlot && fp.active && fp.genid < fc->genid && !(fp.fflags & DP_FLOW_INITIATOR)) {
      if (fp.fflags & dpf::kFlagMasq) gate_vni = fp.dst_vni;
      else if (fp.fflags & dpf::kFlagPf) gate = 1;
    }
  }
  const int t = H.net == 4 ? 0 : 1;
  uint32_t dvni = 0, dnat = 0;
  int32_t pi = -1;
  uint8_t proto = 0;
  Key128 src{0, 0};
  if (!byp) {
  if (H.net == 0) { done(S, DP_DONE_NOT_IP); return; }
  if (!S.src_vni) { done(S, DP_DONE_UNROUTABLE); return; }
  proto = net_proto(F, H);
  src = key_of(F, H, S, true);
  const Key128 dst = key_of(F, H, S, false);
  const auto &VR = VNI_REC(S.vni_idx);
  int32_t rg = VR.ffr[t];
  // v4 candidate-list group: walk its index straight from the VNI context
  uint32_t pre = (t == 0 && VR.ffr4.root) ? mbi_walk(g, VR.ffr4, mbi_key(S, VR.ffr4.field, false) *
                                                                    (VR.ffr4.field & 1))
                                          : NO_PRE;
  if (gate_vni) {  // the (src, GateVni) group: no hoisted walk, the classifier walks it
    uint32_t gi;
    rg = hash_find(g, g.im.ff_remote[t].groups, S.src_vni, gate_vni, 0, gi) ? (int32_t)gi : -1;
    pre = NO_PRE;
  }
  const Hit rh = classify<W_ACTION | W_ACTION2 | W_AUX>(g, CLS_ARRAYS(ff_remote, t), rg, t, proto,
                                                       Key128{0, 0}, dst, 0, S.dport, pre);
  if (rh.rule < 0) {
    if constexpr (FL) if (fp.slot != dpf::kNoSlot) fp.ev0 = fp.slot;
    done(S, DP_DONE_FILTERED);
    return;
  }
  dvni = rh.action;
  dnat = rh.action2;
  pi = (int32_t)rh.aux;
  TRIP_ST(3);
  TRIP();
  } else {
    pi = pair_of(g, S);
  }
  if (t == 0 && pi >= 0) hoist_walks(g, S, pi, P);
  if (byp) return;
  int32_t lg = CTX_TAB(PairRec, g.im.ctx_prec, g.im.pair_recs)[pi].ffl[t];
  uint32_t lpre = P.ffl;
  if (gate) {  // the (src, dst, PortFwdReply) group: no hoisted walk, the classifier walks it
    uint32_t gi;
    lg = hash_find(g, g.im.ff_local[t].groups, S.src_vni, dvni, gate, gi) ? (int32_t)gi : -1;
    lpre = NO_PRE;
  }
  const Hit lh = classify<W_ACTION>(g, CLS_ARRAYS(ff_local, t), lg, t, proto, src, Key128{0, 0}, S.sport, 0, lpre);
  if (lh.rule < 0) {
    if constexpr (FL) if (fp.slot != dpf::kNoSlot) fp.ev0 = fp.slot;
    done(S, DP_DONE_FILTERED);
    return;
  }
  uint32_t snat = lh.action;
  S.dst_vni = dvni;
  S.pair = pi;
  // set_nat_requirements (lib.rs:233-246)
  if (snat == DP_NAT_STATIC) S.flags |= DP_META_REQ_STATIC_NAT_SRC;
  if (dnat == DP_NAT_STATIC) S.flags |= DP_META_REQ_STATIC_NAT_DST;
  if (SNAT && (snat == DP_NAT_PORT_FORWARDING || dnat == DP_NAT_PORT_FORWARDING)) S.flags |= DP_META_REQ_PORT_FORWARDING;
  if (SNAT && (snat == DP_NAT_MASQUERADE || dnat == DP_NAT_MASQUERADE)) S.flags |= DP_META_REQ_MASQUERADE;
  if constexpr (FL) {
    // the key before static NAT, for the flow pair port forwarding or
    // masquerade creates (lib.rs:193-201): recorded in the packet's NAT record
#ifndef DP_X_NOIKEY
    if (SNAT && (S.flags & (DP_META_REQ_PORT_FORWARDING | DP_META_REQ_MASQUERADE)) &&
        (S.flags & (DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST)) && !fc->replay) {
      dpf::FKey k;
      if (packet_fkey(F, H, S, k)) {
        fp.pf_rec = wave_claim(&fc->pf_cnt[0], true);
        dpf::PfReq *R = fc->pf + fp.pf_rec;
#pragma unroll
        for (int j = 0; j < 11; j++) R->ikey[j] = k.w[j];
        R->bits = dpf::kPqIkey;
      }
    }
#endif
    // should_invalidate_flow (lib.rs:258-294): a flow of another generation
    // is outdated if its destination or its NAT requirements differ, or if
    // it no longer needs state
    if (fp.slot != dpf::kNoSlot && fp.genid != fc->genid) {
      const bool pf = SNAT && (S.flags & DP_META_REQ_PORT_FORWARDING), need_pf = SNAT && (fp.fflags & dpf::kFlagPf);
      const bool mq = SNAT && (S.flags & DP_META_REQ_MASQUERADE), need_mq = SNAT && (fp.fflags & dpf::kFlagMasq);
      if (fp.dst_vni != dvni || mq != need_mq || pf != need_pf || (!pf && !mq)) fp.ev0 = fp.slot;
    }
  }
}

// AclFilter (acl-filter/src/lib.rs:51-138).  The classifier action word
// carries the verdict (low byte) and the rule's AclScope (dp_tables.cpp).
// FL: a direct miss with a valid attached flow (active, not outdated:
// packet_has_valid_flow :71-94) whose related flow is in the table looks up
// the related flow's key between the swapped VPCs (reverse_summary
// :205-217); a Flow-scope Allow there admits the packet (:110-128).  That
// verdict rests on the flow still being valid when the packet reaches the
// ACL -- an invalidation by the flow filter (any packet of the burst) or by
// an earlier packet's deny turns it into the peering default
// (dp_flow_fixup).  A deny invalidates the packet's flow pair.
// The replay pass (rp: the packet's port-forwarding record) takes a flow-
// dependent verdict from the first pass, as dp_nat_resolve left it.
template <bool FL>
__device__ __forceinline__ void stage_acl(const Img &g, const Frame &F, const Hdr &H, State &S, const Pre &P,
                                          FlowPk &fp, const dpf::FlowCtx *fc, uint32_t idx,
                                          const dpf::PfReq *rp) {
  if (S.done != DONE_NONE || !(S.flags & DP_META_IS_OVERLAY)) return;
  if (!S.src_vni || !S.dst_vni) { done(S, DP_DONE_UNROUTABLE); return; }
  if (H.net == 0) { done(S, DP_DONE_NOT_IP); return; }
  if constexpr (FL) {
    if (rp) {
      // the replay: the first pass's outcome from the record, no classifier
      // walk -- for a packet whose verdict rests on a flow (verdict 6), the
      // peering default unless the NAT pass kept the flow valid (acl_over 0)
      uint32_t action;
      if (rp->bits & dpf::kPqSens) {
        const uint32_t def = rp->acl_def;
        S.acl = (uint8_t)def;
        action = def == 4 ? DP_ACL_DENY : DP_ACL_ALLOW;
        if (rp->acl_over == 0) {
          action = DP_ACL_ALLOW;
          S.acl = 6;
          S.acl_rule = rp->acl_rule6;
        }
      } else {
        S.acl = (uint8_t)rp->acl_code;
        S.acl_rule = rp->acl_rule;
        action = (S.acl == 2 || S.acl == 4) ? DP_ACL_DENY : DP_ACL_ALLOW;
      }
      if (action == DP_ACL_DENY) done(S, DP_DONE_ACL_DROPPED);
      return;
    }
  }
  uint8_t proto = net_proto(F, H);
  int t = H.net == 4 ? 0 : 1;
  const int32_t pi = pair_of(g, S);
  const int32_t ag = pi >= 0 ? CTX_TAB(PairRec, g.im.ctx_prec, g.im.pair_recs)[pi].acl[t] : -1;
  const Hit ah = classify<W_ACTION | W_ORIG>(g, CLS_ARRAYS(acl, t), ag, t, proto, key_of(F, H, S, true),
                                             key_of(F, H, S, false), S.sport, S.dport, t == 0 ? P.acl : NO_PRE);
  uint32_t action;
  if (ah.rule >= 0) {
    action = ah.action & 0xffu;
    S.acl_rule = ah.orig;
    S.acl = action == DP_ACL_DENY ? 2 : 1;
  } else {
    uint32_t v = pi >= 0 ? CTX_TAB(PairRec, g.im.ctx_prec, g.im.pair_recs)[pi].acl_def : 0;
    const uint8_t def = v ? ((v - 1) == DP_ACL_DENY ? 4 : 3) : 5;
    action = v ? v - 1 : DP_ACL_ALLOW;
    S.acl = def;
    if constexpr (FL) {
      if (!rp && fp.slot != dpf::kNoSlot && fp.active && fp.genid >= fc->genid && fp.related <= fc->mask) {
        const dpf::FlowSlot *r = fc->slots + fp.related;
        const uint4 a = ld4(&r->state), b = ld4(&r->src[0]), c = ld4(&r->dst[0]);
        if (a.x == fp.related_tag) {  // the related flow is still in the table (Weak::upgrade)
        const uint32_t fam = a.z & 0xffu, kind = a.z >> 8;
        const bool ports = kind == DP_FLOW_TCP || kind == DP_FLOW_UDP;
        const uint8_t rproto = kind == DP_FLOW_TCP ? 6 : kind == DP_FLOW_UDP ? 17 : fam == 4 ? 1 : 58;
        const int rt = fam == 4 ? 0 : 1;
        uint32_t rpi;
        const int32_t rg = pair_find(g, S.dst_vni, S.src_vni, rpi)
                               ? CTX_TAB(PairRec, g.im.ctx_prec, g.im.pair_recs)[rpi].acl[rt] : -1;
        Key128 ks, kd;
        if (fam == 4) {
          ks = Key128{0, __builtin_bswap32(b.x)};
          kd = Key128{0, __builtin_bswap32(c.x)};
        } else {
          ks = Key128{((uint64_t)__builtin_bswap32(b.x) << 32) | __builtin_bswap32(b.y),
                      ((uint64_t)__builtin_bswap32(b.z) << 32) | __builtin_bswap32(b.w)};
          kd = Key128{((uint64_t)__builtin_bswap32(c.x) << 32) | __builtin_bswap32(c.y),
                      ((uint64_t)__builtin_bswap32(c.z) << 32) | __builtin_bswap32(c.w)};
        }
        const Hit rh = classify<W_ACTION | W_ORIG>(g, CLS_ARRAYS(acl, rt), rg, rt, rproto, ks, kd,
                                                   ports ? (uint16_t)(a.w >> 16) : 0,
                                                   ports ? (uint16_t)a.w : 0);
        if (rh.rule >= 0 && rh.action == (DP_ACL_ALLOW | (DP_ACL_SCOPE_FLOW << 8))) {
          action = DP_ACL_ALLOW;
          S.acl = 6;
          S.acl_rule = rh.orig;
          fp.sens = true;
          fp.def_acl = def;
          fp.s_flags = S.flags;
          fp.s_oif = S.has_oif ? S.oif : 0;
          fp.s_fib = S.fib_entry;
          fp.s_dvni = S.dst_vni;
          fp.s_vrf = S.has_vrf ? (0x80000000u | S.vrf) : 0u;
          fp.s_nh = S.nh_ref;
          fp.acl_rule6 = rh.orig;
        }
        }
      }
    }
  }
  if (action == DP_ACL_DENY) {
    if constexpr (FL) if (fp.slot != dpf::kNoSlot && !rp) { fp.ev1 = fp.slot; fp.ev_mark = idx + 1; }
    done(S, DP_DONE_ACL_DROPPED);
  }
}

// The NAT record of a packet that reached PortForwarder or Masquerade in the
// first pass (dpf::PfReq): what the sequential NAT pass (dp_nat_resolve) needs
// to run the reference's NFs over it in packet order.  The packet stops here;
// the replay pass finishes it with the pass's decisions.
__device__ __forceinline__ void nat_record(const Frame &F, const Hdr &H, const State &S, FlowPk &fp,
                                           const dpf::FlowCtx *fc, uint32_t idx) {
  const uint32_t claim = wave_claim(&fc->pf_cnt[0], fp.pf_rec == dpf::kNoSlot);
  const uint32_t rec = fp.pf_rec != dpf::kNoSlot ? fp.pf_rec : claim;
  dpf::PfReq *R = fc->pf + rec;
  uint32_t bits = (fp.pf_rec != dpf::kNoSlot ? R->bits : 0u) | dpf::kPqReached | dpf::kPqEth;
  if (S.flags & DP_META_REQ_PORT_FORWARDING) bits |= dpf::kPqPf;
  if (S.flags & DP_META_REQ_MASQUERADE) bits |= dpf::kPqMasq;
  if (H.l4 == L4_TCP) bits |= dpf::kPqTcp;
  if (H.l4 == L4_UDP) bits |= dpf::kPqUdp;
  if (H.l4 == L4_ICMP4 || H.l4 == L4_ICMP6) {
    bits |= dpf::kPqIcmp;
    // IcmpProtoKey::new_icmp_v4/v6 (flow_key.rs:318-338): Echo Request / Reply
    const uint8_t t = F.b(H.l4_off), c = F.b(H.l4_off + 1);
    if (c == 0 && (H.l4 == L4_ICMP6 ? (t == 128 || t == 129) : (t == 0 || t == 8))) bits |= dpf::kPqQuery;
  }
  if (fp.sens) bits |= dpf::kPqSens;
  if (S.flags & DP_META_REQ_STATIC_NAT_SRC) bits |= dpf::kPqSnatSrc;
  if (S.flags & DP_META_REQ_STATIC_NAT_DST) bits |= dpf::kPqSnatDst;
  R->idx = idx;
  R->slot = fp.slot;
  R->state = fp.state;
  if (fp.slot != dpf::kNoSlot) {
    bits |= dpf::kPqRelated;
    R->status0 = fp.active ? DP_FLOW_ACTIVE : DP_FLOW_CANCELLED;
    R->fflags0 = fp.fflags;
    R->dst_vni0 = fp.dst_vni;
    R->related0 = fp.related;
    R->related_tag0 = fp.related_tag;
    R->genid0 = fp.genid;
  }
  R->bits = bits;
  R->src_vni = S.src_vni;
  R->dst_vni = S.dst_vni;
  const uint32_t tflags = H.l4 == L4_TCP ? F.b(H.l4_off + 13) : 0u;
  R->proto = (uint32_t)net_proto(F, H) | ((uint32_t)H.net << 8) | (tflags << 16);
  // TCP / UDP ports; an ICMP query's identifier (its flow key's)
  R->ports = (bits & dpf::kPqQuery) ? be16_bytes(F, H.l4_off + 4) << 16 : ((uint32_t)S.sport << 16) | S.dport;
  if (H.net == 4) {
    R->src[0] = S.v4src; R->dst[0] = S.v4dst;
    R->src[1] = R->src[2] = R->src[3] = R->dst[1] = R->dst[2] = R->dst[3] = 0;
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      R->src[j] = F.be32(H.net_off + 8 + 4 * j);
      R->dst[j] = F.be32(H.net_off + 24 + 4 * j);
    }
  }
  R->acl_def = fp.def_acl;
  R->acl_rule6 = fp.acl_rule6;
  R->acl_code = S.acl;
  R->acl_rule = S.acl_rule;
  R->acl_over = 0;
  fc->pf_of[idx] = rec;  // (its bit in the burst's bitmap: flow_effects, per wave)
  fp.pf_rec = rec;
  fp.deferred = true;
}

__device__ __forceinline__ bool icmp_error_pkt(const Frame &F, const Hdr &H) {
  return (H.l4 == L4_ICMP4 || H.l4 == L4_ICMP6) && icmp_err_at(F, H.l4_off, H.l4 == L4_ICMP6);
}

// PortForwarder (nat/src/portfw/nf.rs:373-397) for a packet that requires
// port forwarding and is not an ICMP error.  Its outcome depends on the flow
// states the earlier packets of the burst leave (NatFlowStatus, expiry,
// invalidations, the flow pairs they create), so the first pass records the
// packet (nat_record) and stops it here; dp_nat_resolve runs the reference's
// PortForwarder over the records in packet order, and the replay pass takes
// each packet through the rest of the path with its decision.  Without a
// flow table (whose Arc the reference's PortForwarder always holds) the
// stage fails the packet.
template <bool FL>
__device__ __forceinline__ void stage_portfw(const Frame &F, const Hdr &H, State &S, FlowPk &fp,
                                             const dpf::FlowCtx *fc, uint32_t idx, const dpf::PfReq *rp) {
  if (S.done != DONE_NONE || !(S.flags & DP_META_REQ_PORT_FORWARDING)) return;
  if (icmp_error_pkt(F, H)) return;
  if constexpr (!FL) {
    done(S, DP_DONE_INTERNAL_FAILURE);
  } else if (!rp) {
#ifdef DP_X_NOREC
    fp.deferred = true; return;
#endif
    nat_record(F, H, S, fp, fc, idx);
  } else {
    // a flow pair refused at capacity was translated before the inserts
    // (do_port_forwarding, nf.rs:142-163): its metadata says so
    const uint32_t v = rp->verdict;
    if (v != dpf::kPfForward && v != DP_DONE_FLOW_CAPACITY_EXCEEDED) { done(S, (uint8_t)v); return; }
    // nat_packet (portfw/packet.rs:42-154): address and port of the side the
    // action names, each only if it changes
    const bool src = (rp->nat & 0xffu) == DP_PF_SRC_NAT;
    const uint16_t port = (uint16_t)(rp->nat >> 16);
    bool mod = false;
    if (H.net == 4) {
      uint32_t &a = src ? S.v4src : S.v4dst;
      if (a != rp->nat_ip[0]) { a = rp->nat_ip[0]; mod = true; }
    } else {
      const int oo = H.net_off + (src ? 8 : 24);
      for (int j = 0; j < 4; j++)
        if (F.be32(oo + 4 * j) != rp->nat_ip[j]) { wput32(F, oo + 4 * j, rp->nat_ip[j]); mod = true; }
    }
    if (H.l4 == L4_TCP || H.l4 == L4_UDP) {
      uint16_t &pp = src ? S.sport : S.dport;
      if (pp != port) { pp = port; mod = true; }
    }
    if (mod) S.flags |= DP_META_REFR_CHKSUM | (src ? DP_META_NATTED_SRC : DP_META_NATTED_DST);
    if (v != dpf::kPfForward) done(S, (uint8_t)v);
  }
}

// Masquerade (nat/src/masquerade/nf.rs:511-586) for a packet that requires
// masquerading and is not an ICMP error: like PortForwarder, its outcome
// rests on what the earlier packets of the burst did to the flows and to the
// allocator, so the first pass records it (one record with PortForwarder's
// when the packet needs both) and dp_nat_resolve decides.  The replay applies
// the decision: masquerade (packet.rs:35-195) -- the address, a TCP / UDP
// port always, an ICMP query identifier when it changes -- and the checksum
// refresh the NF always asks for.  Without a flow table: InternalFailure.
template <bool FL>
__device__ __forceinline__ void stage_masquerade(const Frame &F, const Hdr &H, State &S, FlowPk &fp,
                                                 const dpf::FlowCtx *fc, uint32_t idx, const dpf::PfReq *rp) {
  if (S.done != DONE_NONE || !(S.flags & DP_META_REQ_MASQUERADE)) return;
  if (icmp_error_pkt(F, H)) return;
  if constexpr (!FL) {
    done(S, DP_DONE_INTERNAL_FAILURE);
  } else if (!rp) {
    if (!fp.deferred) nat_record(F, H, S, fp, fc, idx);
  } else {
    const uint32_t v = rp->mverdict;
    if (v != dpf::kPfForward) { done(S, (uint8_t)v); return; }
    const bool src = (rp->mnat & 0xffu) == DP_PF_SRC_NAT, ident = rp->mnat & 0x100u;
    const uint16_t port = (uint16_t)(rp->mnat >> 16);
    bool mod = false;
    if (H.net == 4) {
      uint32_t &a = src ? S.v4src : S.v4dst;
      if (a != rp->mnat_ip[0]) { a = rp->mnat_ip[0]; mod = true; }
    } else {
      const int oo = H.net_off + (src ? 8 : 24);
      for (int j = 0; j < 4; j++)
        if (F.be32(oo + 4 * j) != rp->mnat_ip[j]) { wput32(F, oo + 4 * j, rp->mnat_ip[j]); mod = true; }
    }
    if (H.l4 == L4_TCP || H.l4 == L4_UDP) {
      if (!ident) {  // NatPort::Port: set, changed or not
        (src ? S.sport : S.dport) = port;
        mod = true;
      }
    } else if (ident) {
      // an ICMP query's identifier (icmp_full_identifier: v4 echo / timestamp,
      // v6 echo, code 0), only if it changes
      const uint8_t t = F.b(H.l4_off), c = F.b(H.l4_off + 1);
      const bool q = c == 0 && (H.l4 == L4_ICMP6 ? (t == 128 || t == 129) : (t == 0 || t == 8 || t == 13 || t == 14));
      if (q && F.be16(H.l4_off + 4) != port) {
        wput16(F, H.l4_off + 4, port);
        mod = true;
      }
    }
    if (mod) S.flags |= src ? DP_META_NATTED_SRC : DP_META_NATTED_DST;
    S.flags |= DP_META_REFR_CHKSUM;
  }
}

// The embedded packet of an ICMP error message, translated back by static
// NAT (nat/src/static_nat/nf.rs:111-155, nat/src/icmp_handler/
// icmp_error_msg.rs nat_translate_icmp_inner_src/dst): its destination
// through the source table (find_src_mapping), its source through the
// destination table (find_dst_mapping), with the ports of a TCP / UDP
// header (full or partial).  q[0]: inner destination, q[1]: inner source.
// Returns false without an embedded IPv4 header.
__device__ __forceinline__ bool nat_icmp_inner(const Img &g, const Frame &F, const Hdr &H, int32_t st, int32_t dt, NatQ q[2],
                                               EmbV &E) {
  E = emb_view(F, H);
  if (E.net != 4) return false;
  const bool hp = E.tk == L4_TCP || E.tk == L4_UDP;
  q[0].ti = st; q[0].addr = F.be32(E.off + 16); q[0].port = hp ? F.be16(E.t_off + 2) : 0;
  q[1].ti = dt; q[1].addr = F.be32(E.off + 12); q[1].port = hp ? F.be16(E.t_off) : 0;
  const uint32_t pre[2] = {NO_PRE, NO_PRE};
  nat_find2(g, q, hp, pre);
  return true;
}

__device__ __forceinline__ void stage_static_nat(const Img &g, const Frame &F, const Hdr &H, State &S, const Pre &P) {
  if (S.done != DONE_NONE) return;
  if (!(S.flags & (DP_META_REQ_STATIC_NAT_SRC | DP_META_REQ_STATIC_NAT_DST))) return;
  // an ICMP error message with an embedded packet is translated even when
  // already marked NATed (nf.rs:350-362)
  const bool ie = has_emb(H) && icmp_err_at(F, H.l4_off, H.l4 == L4_ICMP6);
  if ((S.flags & (DP_META_NATTED_SRC | DP_META_NATTED_DST)) && !ie) return;
  if (!S.src_vni || !S.dst_vni) { done(S, DP_DONE_UNROUTABLE); return; }
  const auto &VR = VNI_REC(S.vni_idx);
  if (!VR.pervni) { done(S, DP_DONE_UNROUTABLE); return; }
  if (H.net == 0) { done(S, DP_DONE_NOT_IP); return; }
  const int32_t pi = pair_of(g, S);
  const int32_t st = pi >= 0 ? CTX_TAB(PairRec, g.im.ctx_prec, g.im.pair_recs)[pi].nat_src : -1;
  bool has_p = H.l4 == L4_TCP || H.l4 == L4_UDP;
  bool modified = false;
  NatQ q[2];
  q[0].ti = (H.net == 4 && (S.flags & DP_META_REQ_STATIC_NAT_SRC)) ? st : -1;
  q[0].addr = S.v4src; q[0].port = has_p ? S.sport : 0;
  q[1].ti = (H.net == 4 && (S.flags & DP_META_REQ_STATIC_NAT_DST)) ? VR.nat_dst : -1;
  q[1].addr = S.v4dst; q[1].port = has_p ? S.dport : 0;
  const uint32_t pre[2] = {P.nsrc, P.ndst};
  nat_find2(g, q, has_p, pre);
  NatQ qi[2];
  EmbV E;
  const bool inner = ie && nat_icmp_inner(g, F, H, st, VR.nat_dst, qi, E);
  const bool inner_p = inner && (E.tk == L4_TCP || E.tk == L4_UDP);
  if ((S.flags & DP_META_REQ_STATIC_NAT_SRC) && !(S.flags & DP_META_NATTED_SRC)) {
    bool mod = false;
    // source mapping: UnicastIpAddr::try_from rejects multicast / broadcast
    if (q[0].ok && !((q[0].na >> 28) == 0xe || q[0].na == 0xffffffffu)) {
      if (q[0].na != S.v4src) { S.v4src = q[0].na; mod = true; }
      if (has_p && q[0].hp && q[0].np != S.sport) { S.sport = q[0].np; mod = true; }
    }
    // the embedded destination (find_src_mapping: unicast only); a mapping
    // found counts as a modification (Ok(true))
    if (inner && qi[0].ok && !((qi[0].na >> 28) == 0xe || qi[0].na == 0xffffffffu)) {
      wput32(F, E.off + 16, qi[0].na);
      if (inner_p && qi[0].hp) wput16(F, E.t_off + 2, qi[0].np);
      mod = true;
    }
    if (mod) S.flags |= DP_META_NATTED_SRC;
    modified |= mod;
  }
  if ((S.flags & DP_META_REQ_STATIC_NAT_DST) && !(S.flags & DP_META_NATTED_DST)) {
    bool mod = false;
    if (q[1].ok) {
      if (q[1].na != S.v4dst) { S.v4dst = q[1].na; mod = true; }
      if (has_p && q[1].hp && q[1].np != S.dport) { S.dport = q[1].np; mod = true; }
    }
    // the embedded source (find_dst_mapping): a non-unicast target is
    // NotUnicast -> NatFailure
    if (inner && qi[1].ok) {
      if ((qi[1].na >> 28) == 0xe || qi[1].na == 0xffffffffu) { done(S, DP_DONE_NAT_FAILURE); return; }
      wput32(F, E.off + 12, qi[1].na);
      if (inner_p && qi[1].hp) wput16(F, E.t_off, qi[1].np);
      mod = true;
    }
    if (mod) S.flags |= DP_META_NATTED_DST;
    modified |= mod;
  }
  if (modified) S.flags |= DP_META_REFR_CHKSUM;
}

__device__ __forceinline__ bool adj_find(const Img &g, uint32_t oif, uint8_t fam, const Addr16 &a, uint8_t mac[6]) {
  const AdjMap &m = g.im.adjs;
  if (m.count == 0) return false;
  const Adj *s = g.at<Adj>(m.slots);
  uint32_t h = hmix(oif ^ (fam << 24), a.w[0] ^ a.w[2], a.w[1] ^ a.w[3]) & m.mask;
  for (uint32_t probe = 0; probe <= m.mask; probe++) {
    const Adj &e = s[h];
    if (!e.used) return false;
    if (e.ifindex == oif && e.fam == fam) {
      // fully unrolled: a constant index keeps `a` in registers (a dynamic
      // a.w[i >> 2] would put it in scratch memory)
      bool eq = true;
      const int n = fam == 4 ? 4 : 16;
#pragma unroll
      for (int i = 0; i < 16; i++)
        if (i < n) eq &= e.addr[i] == (uint8_t)(a.w[i >> 2] >> (24 - 8 * (i & 3)));
      if (eq) {
#pragma unroll
        for (int i = 0; i < 6; i++) mac[i] = e.mac[i];
        return true;
      }
    }
    h = (h + 1) & m.mask;
  }
  return false;
}

__device__ __forceinline__ void stage_egress(const Img &g, const Frame &F, const Hdr &H, State &S) {
  if (S.done != DONE_NONE) return;
  if (!S.has_oif) { done(S, DP_DONE_ROUTE_FAILURE); return; }
  uint64_t dmac = S.eg_dmac;
  if (S.eg_code == DPD_EG_NEED_ADJ) {
    // no next-hop address: adjacency of the packet's (current) destination
    if (!S.encap && !H.net) { done(S, DP_DONE_NOT_IP); return; }
    uint8_t fam; uint64_t khi, klo;
    cur_dst_key(F, H, S, fam, khi, klo);
    const Addr16 a{{(uint32_t)(khi >> 32), (uint32_t)khi, (uint32_t)(klo >> 32), (uint32_t)klo}};
    uint8_t m[6];
    if (!adj_find(g, S.oif, fam, a, m)) { done(S, DP_DONE_MISS_L2_RESOLUTION); return; }
    dmac = load_mac(m);
    if (dmac == 0) { done(S, DP_DONE_INVALID_DST_MAC); return; }
    if (S.if_code != 255) { done(S, S.if_code); return; }
  } else if (S.eg_code != DP_DONE_DELIVERED) {
    done(S, S.eg_code);
    return;
  }
  if (S.encap) {
    S.o_eth = true;
    S.odst = dmac;
    S.osrc = S.eg_smac;
  } else {
    S.edst = dmac;
    S.esrc = S.eg_smac;
    S.eth_dirty = true;
  }
  done(S, DP_DONE_DELIVERED);
}

// ---------------------------------------------------------------------------
// Serialize
// ---------------------------------------------------------------------------
// word i of an address without a dynamic register index (keeps it out of scratch)
__device__ __forceinline__ uint32_t aw(const Addr16 &a, int i) {
  return i == 0 ? a.w[0] : i == 1 ? a.w[1] : i == 2 ? a.w[2] : a.w[3];
}

// outer IPv4 header checksum (0 for an IPv6 outer header)
__device__ __forceinline__ uint32_t outer_ck4(const OuterHdr &S) {
  if (S.fam != 4) return 0;
  uint64_t t = 0x4500u | S.tos;
  t += (uint16_t)(20 + S.len); t += 0x4000; t += (64u << 8) | 17;
  t += (S.src.w[0] >> 16) + (S.src.w[0] & 0xffff) + (S.dst.w[0] >> 16) + (S.dst.w[0] & 0xffff);
  return (uint16_t)~fold(t);
}

// --- serializer ------------------------------------------------------------
__device__ __forceinline__ void wput_mac(const Frame &F, int f, uint64_t m) {
  wput16(F, f, (uint32_t)(m >> 32)); wput32(F, f + 2, (uint32_t)m);
}

// Window positions [p, we) of one slab back to the burst buffer (gbase: the
// 16-aligned address of window position 0; p 16-aligned).
__device__ __forceinline__ void flush_range(uint8_t *gbase, const lds_u8 *slab, int p, int we) {
  const lds_u32 *w = reinterpret_cast<const lds_u32 *>(slab);
#pragma unroll 1
  for (; p + 16 <= we; p += 16)
    *reinterpret_cast<uint4 *>(gbase + p) = make_uint4(w[p >> 2], w[(p >> 2) + 1], w[(p >> 2) + 2], w[(p >> 2) + 3]);
#pragma unroll 1
  for (; p + 4 <= we; p += 4) *reinterpret_cast<uint32_t *>(gbase + p) = w[p >> 2];
#pragma unroll 1
  for (; p < we; p++) gbase[p] = slab[p];
}

// The frame lies inside the burst buffer behind its headroom (else the
// packet is InternalFailure and nothing of it is touched).
__device__ __forceinline__ bool frame_ok(const dp_pkt_in_t &pin, uint64_t buf_bytes) {
  return pin.off >= DP_HEADROOM && (((uint64_t)pin.off + pin.len + 15) & ~15ull) <= buf_bytes;
}
// 16-byte chunks of the header window (the frame's first WIN - shift bytes)
__device__ __forceinline__ int window_chunks(const dp_pkt_in_t &pin) {
  const int c = ((int)(pin.off & 15) + pin.len + 15) >> 4;
  return c < WIN / 16 ? c : WIN / 16;
}

// Packet::serialize (net/src/packet/mod.rs:342-374): deparse the current
// header stack in front of the payload (Headers::deparse), with
// update_checksums (net/src/headers/mod.rs:894-929) -- or, for a VXLAN
// encapsulation, the inner checksums of IpForwarder::vxlan_encap and the
// outer Eth/IP/UDP/VXLAN headers.  Fields are patched into the LDS window
// copy, checksums summed over the patched bytes, and the stack written back
// in 16-byte chunks.  Returns the frame-relative output start.
// The common shape -- the whole frame in the LDS window, no encap / VXLAN /
// extension headers / ICMP error / parse-limit relocation, IPv4 or IPv6 with
// UDP or TCP -- straight-line: the same bytes as the general serialize below,
// with the IPv4 header checksum summed from the field values instead of a
// pass over the patched header.
__device__ __forceinline__ int serialize_fast(const Frame &F, const Hdr &H, const State &S, int &fl0, int &fl1) {
  const int n = H.net_off, l = H.l4_off;
  if (S.eth_dirty) { wput_mac(F, H.hb, S.edst); wput_mac(F, H.hb + 6, S.esrc); }
  uint64_t t;
  if (H.net == 4) {
    const uint32_t w3 = F.be16(n + 6) & 0x7fffu;                 // reserved flag bit not kept
    const uint32_t w4 = ((uint32_t)S.ttl << 8) | F.b(n + 9);
    const uint32_t a = (S.v4src >> 16) + (S.v4src & 0xffff) + (S.v4dst >> 16) + (S.v4dst & 0xffff);
    uint64_t s = (uint64_t)F.be16(n) + F.be16(n + 2) + F.be16(n + 4) + w3 + w4 + a;
    for (int i = 20; i < H.net_hlen; i += 2) s += F.be16(n + i);  // options
    wput16(F, n + 6, w3);
    wput16(F, n + 8, w4);
    wput16(F, n + 10, (uint16_t)~fold(s));
    wput32(F, n + 12, S.v4src);
    wput32(F, n + 16, S.v4dst);
    t = a;
  } else {
    wput8(F, n + 7, S.ttl);
    t = sum_frame(F, n + 8, n + 40);
  }
  wput16(F, l, S.sport);
  wput16(F, l + 2, S.dport);
  const bool udp = H.l4 == L4_UDP;
  if (!udp) wput8(F, l + 12, F.b(l + 12) & 0xf1);
  const int ck_off = udp ? l + 6 : l + 16;
  wput16(F, ck_off, 0);
  t += sum_frame(F, l, F.len);
  const uint32_t tl = (uint32_t)H.l4_hlen + (uint32_t)(F.len - S.pay_start);
  t += udp ? 17u + F.be16(l + 4) : (tl >> 16) + (tl & 0xffff) + 6u;
  uint16_t c = (uint16_t)~fold(t);
  if (udp && c == 0) c = 0xffff;
  wput16(F, ck_off, c);
  const int p = (F.shift + H.hb) & ~15;
  int we = (F.shift + H.hb + H.size + 15) & ~15;
  if (we > F.shift + F.len) we = F.shift + F.len;
  fl0 = fl1 = 0;
  if (we > p) { fl0 = p; fl1 = we; }
  return H.hb;
}

__device__ __forceinline__ int serialize(const Frame &F, Hdr &H, State &S, int &fl0, int &fl1) {
  if (F.inwin && !S.encap && !H.vx && H.next == 0 && !has_emb(H) && S.pay_start - H.size == H.hb &&
      (H.net == 4 || H.net == 6) && (H.l4 == L4_UDP || H.l4 == L4_TCP))
    return serialize_fast(F, H, S, fl0, fl1);
  fl0 = fl1 = 0;
  const int inner_start = S.pay_start - H.size;
  const int outer = S.encap ? 14 + (S.o_fam == 4 ? 20 : 40) + 16 : 0;
  const int start = inner_start - outer;
  if (start < -(int)DP_HEADROOM) { S.done = DP_DONE_NO_HEAD_ROOM; return 0; }
  // the parse-limit quirk consumed headers it did not record: the kept
  // stack moves sh bytes later to end at the payload (back to front)
  const int sh = inner_start - H.hb;
  if (sh) {
#pragma unroll 1
    for (int i = H.size - 1; i >= 0; i--) wput8(F, H.hb + sh + i, F.b(H.hb + i));
    H.hb += sh; H.net_off += sh; H.l4_off += sh; H.vx_off += sh;
#pragma unroll
    for (int e = 0; e < 3; e++) H.ext_off[e] += sh;
  }
  // deparse: rewritten fields and normalised reserved bits
  if (S.eth_dirty) { wput_mac(F, H.hb, S.edst); wput_mac(F, H.hb + 6, S.esrc); }
  if (H.net == 4) {
    const int n = H.net_off;
    wput8(F, n + 6, F.b(n + 6) & 0x7f);
    wput8(F, n + 8, S.ttl);
    wput16(F, n + 10, 0);
    wput32(F, n + 12, S.v4src);
    wput32(F, n + 16, S.v4dst);
  } else if (H.net == 6) {
    wput8(F, H.net_off + 7, S.ttl);
  }
#pragma unroll
  for (int e = 0; e < 3; e++) {
    if (e >= H.next) break;
    const int x = H.ext_off[e];
    if (H.ext_kind[e] == HK_EXT_FRAG) { wput8(F, x + 1, 0); wput8(F, x + 3, F.b(x + 3) & 0xf9); }
    if (H.ext_kind[e] == HK_EXT_AUTH) { wput16(F, x + 2, 0); }
  }
  // L4 checksum: recomputed unless VXLAN (outer) or, for an encapsulated
  // inner stack, REFR_CHKSUM was clear at encap
  const bool l4 = H.net && H.l4 != L4_NONE && !H.vx && (!S.encap || S.inner_l4_ck);
  const int l = H.l4_off;
  int ck_off = -1;
  if (H.net && H.l4) {
    if (H.l4 == L4_TCP || H.l4 == L4_UDP) { wput16(F, l, S.sport); wput16(F, l + 2, S.dport); }
    if (H.l4 == L4_TCP) wput8(F, l + 12, F.b(l + 12) & 0xf1);
    if (l4) {
      ck_off = H.l4 == L4_UDP ? l + 6 : H.l4 == L4_TCP ? l + 16 : l + 2;
      wput16(F, ck_off, 0);
    }
    if (H.vx) wput8(F, H.vx_off, 0x08);
  }
  if (H.net == 4) wput16(F, H.net_off + 10, (uint16_t)~fold(sum_frame(F, H.net_off, H.net_off + H.net_hlen)));
  if (ck_off >= 0 && has_emb(H)) {
    const EmbV E = emb_view(F, H);
    // update_checksums with embedded headers (net/src/headers/mod.rs:906-928):
    // the embedded IPv4 header first (part of the ICMP payload; its transport
    // checksum stays), then the ICMP checksum over get_payload_for_checksum
    if (E.net == 4) wput16(F, E.off + 10, emb_ipv4_ck(F, E));
    wput16(F, ck_off, (uint16_t)~icmp_err_sum(F, H, E, S.pay_start));
  } else if (ck_off >= 0) {
    uint64_t t = sum_frame(F, l, F.len);
    const uint32_t tl = (uint32_t)H.l4_hlen + (uint32_t)(F.len - S.pay_start);
    if (H.l4 != L4_ICMP4) {  // pseudo header
      if (H.net == 4) t += (S.v4src >> 16) + (S.v4src & 0xffff) + (S.v4dst >> 16) + (S.v4dst & 0xffff);
      else t += sum_frame(F, H.net_off + 8, H.net_off + 40);
      if (H.l4 == L4_UDP) t += 17u + F.be16(l + 4);
      else t += (tl >> 16) + (tl & 0xffff) + (H.l4 == L4_TCP ? 6u : 58u);
    }
    uint16_t c = (uint16_t)~fold(t);
    if (H.l4 == L4_UDP && c == 0) c = 0xffff;
    wput16(F, ck_off, c);
  }
  if (S.encap) {  // outer Ethernet (Egress), then the outer IP/UDP/VXLAN deparsed at encap
#pragma unroll
    for (int i = 0; i < 6; i++) {
      wput8_any(F, start + i, mac_b(S.odst, i));
      wput8_any(F, start + 6 + i, mac_b(S.osrc, i));
    }
    wput8_any(F, start + 12, S.o_fam == 4 ? 0x08u : 0x86u);
    wput8_any(F, start + 13, S.o_fam == 4 ? 0x00u : 0xddu);
    const int nb = 2 * (outer_words(S.o_fam) - 7);
#pragma unroll 1
    for (int i = 0; i < nb; i++) wput8_any(F, start + 14 + i, F.hs[i]);
  }
  // write-back range: window positions [fl0, fl1) covering [start, end of
  // the stack), widened to whole 16-byte chunks inside [0, min(frame end,
  // WIN)) -- this packet's own bytes, rewritten with the values read; bytes
  // outside the window went straight to the buffer (wput8)
  int p = F.shift + start;
  p = (p < 0 ? 0 : p) & ~15;
  const int lim = F.shift + F.len < WIN ? F.shift + F.len : WIN;
  int we = (F.shift + H.hb + H.size + 15) & ~15;
  if (we > lim) we = lim;
  if (we > p) { fl0 = p; fl1 = we; }
  return start;
}

// ---------------------------------------------------------------------------
// Burst records
// ---------------------------------------------------------------------------
__device__ __forceinline__ dp_pkt_out_t out_record(uint32_t off, uint16_t len, uint8_t done) {
  dp_pkt_out_t o;
  o.off = off; o.len = len; o.done = done; o.acl = 0; o.oif = 0; o.meta_flags = 0; o.pad = 0;
  return o;
}
// PacketMeta of a packet no stage annotated
__device__ __forceinline__ dp_pkt_meta_t meta_none() {
  dp_pkt_meta_t m;
  m.dst_vni = m.src_vni = 0;
  m.fib_entry = m.acl_rule = 0xffffffffu;
  m.vrf = 0; m.pm_flags = 0; m.dscp = m.ecn = 0; m.nh_family = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) m.nh_addr[i] = 0;
  m.flow_ref = ~0ull;
  return m;
}
// PacketMeta.nh_addr: the address of the last Egress instruction executed
// (packet_exec_instruction_egress, ipforward.rs:308-327: None without one)
__device__ __forceinline__ void meta_nh(const Img &g, uint32_t nh_ref, dp_pkt_meta_t &m) {
  if (nh_ref == NH_NONE) return;
  const uint32_t ii = (nh_ref & NH_ENTRY) ? g.at<Entry>(g.im.entries)[nh_ref & ~NH_ENTRY].first_instr : nh_ref;
  const Instr &in = g.at<Instr>(g.im.instrs)[ii];
  if (!(in.flags & DP_INSTR_HAS_ADDR)) return;
  m.pm_flags |= DP_PM_HAS_NH;
  m.nh_family = in.fam;
#pragma unroll
  for (int i = 0; i < 16; i++) m.nh_addr[i] = in.addr[i];
}
__device__ __forceinline__ dp_pkt_meta_t meta_of(const Img &g, const State &S) {
  dp_pkt_meta_t m = meta_none();
  m.dst_vni = S.dst_vni;
  m.src_vni = S.src_vni;
  m.fib_entry = S.fib_entry;
  m.acl_rule = S.acl_rule;
  if (S.has_vrf) { m.pm_flags |= DP_PM_HAS_VRF; m.vrf = S.vrf; }
  if (S.has_dscp) { m.pm_flags |= DP_PM_HAS_DSCP; m.dscp = S.dscp; m.ecn = S.ecn; }
  meta_nh(g, S.nh_ref, m);
  return m;
}

#ifndef DP_EMU
// The flow-table effects of a wave's packets (FL only), wave-aggregated:
// flow refs, invalidation marks and events, flow-dependent ACL verdicts.
template <bool MT>
__device__ __forceinline__ void flow_effects(const dpf::FlowCtx &fc, bool live, uint32_t i, const FlowPk &fp) {
  const int lane = threadIdx.x & 63;
  const bool has = live && fp.slot != dpf::kNoSlot;
  const bool e0 = has && fp.ev0 != dpf::kNoSlot, e1 = has && fp.ev1 != dpf::kNoSlot;
  const bool e2 = live && fp.ev2 != dpf::kNoSlot;  // an ICMP error's (mark 0, like the flow filter's)
  if (e0) atomicMin(&fc.slots[fp.ev0].mark, 0u);
  if (e1) atomicMin(&fc.slots[fp.ev1].mark, fp.ev_mark);
  if (e2) atomicMin(&fc.slots[fp.ev2].mark, 0u);
  const uint64_t m0 = __ballot(e0), m1 = __ballot(e1), m2 = __ballot(e2);
  if (m2) {
    const int leader = __ffsll((long long)m2) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&fc.events[0], (uint32_t)__popcll(m2));
    base = (uint32_t)__shfl((int)base, leader);
    if (e2) {
      const uint32_t k = base + __popcll(m2 & lanes_below(lane));
      fc.events[1 + 2 * k] = fp.ev2;
      fc.events[2 + 2 * k] = fp.ev2_tag;
    }
  }
  if (m0 | m1) {
    const int leader = __ffsll((long long)(m0 | m1)) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&fc.events[0], (uint32_t)(__popcll(m0) + __popcll(m1)));
    base = (uint32_t)__shfl((int)base, leader);
    // (slot, state word) pairs: the fill of the packet's flow (ev0 / ev1 are fp.slot)
    if (e0) {
      const uint32_t k = base + __popcll(m0 & lanes_below(lane));
      fc.events[1 + 2 * k] = fp.ev0;
      fc.events[2 + 2 * k] = fp.state;
    }
    if (e1) {
      const uint32_t k = base + __popcll(m0) + __popcll(m1 & lanes_below(lane));
      fc.events[1 + 2 * k] = fp.ev1;
      fc.events[2 + 2 * k] = fp.state;
    }
  }
  // the packets recorded for the NAT pass: a wave's 64 packets are the two
  // bitmap words it alone owns (first pass: packet i on lane i % 64), stored
  // whole; the region's summary bit once per wave, read first (a chip's
  // worth of waves on a few summary words would queue at one L2 channel)
  const uint64_t mr = SNAT ? __ballot(live && fp.deferred) : 0ull;
  if (mr && lane == __ffsll((long long)mr) - 1) {
    const uint32_t w0 = (i - lane) >> 5;
    if ((uint32_t)mr) fc.pf_bits[w0] = (uint32_t)mr;
    if (mr >> 32) fc.pf_bits[w0 + 1] = (uint32_t)(mr >> 32);
    uint32_t *sw = &fc.pf_sum[i >> 15];
    const uint32_t sb = 1u << ((i >> 10) & 31);
    if (!(__hip_atomic_load(sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & sb)) atomicOr(sw, sb);
  }
  const bool sv = has && fp.sens && !fp.deferred;  // a deferred packet's verdict: dp_nat_resolve
  const uint64_t ms = __ballot(sv);
  if (ms) {
    const int leader = __ffsll((long long)ms) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&fc.sens[0], (uint32_t)__popcll(ms));
    base = (uint32_t)__shfl((int)base, leader);
    if (sv) {
      dpf::SensRec *R = reinterpret_cast<dpf::SensRec *>(fc.sens + 8) + base + __popcll(ms & lanes_below(lane));
      *R = dpf::SensRec{i, fp.slot, fp.s_flags, fp.s_oif, fp.s_fib, fp.def_acl, fp.related, fp.related_tag,
                        MT ? fp.s_dvni : 0u, MT ? fp.s_vrf : 0u, MT ? fp.s_nh : NH_NONE, fp.state};
    }
  }
}
#endif

// ---------------------------------------------------------------------------
// Per-packet body
// ---------------------------------------------------------------------------
// FL: the flows variant -- FlowLookup on fc's table and the flow-aware
// branches; fp receives the packet's flow and its flow-table effects.
// MT: the caller asked for PacketMeta records (pm); without them the values
// only the meta record carries (vrf, dscp / ecn, nh_ref, ...) are dead and
// the compiler drops them -- the transmit path keeps its registers.
template <bool FL, bool MT>
__device__ __forceinline__ uint8_t process_packet(const Img &g, lds_u8 *slab, lds_u8 *hs, uint8_t *buf, uint64_t buf_bytes,
                                  const dp_pkt_in_t &pin, dp_pkt_out_t &o, dp_pkt_meta_t *pm, int &fl0, int &fl1,
                                  bool inwin, const dpf::FlowCtx *fc, FlowPk &fp, uint32_t idx,
                                  const dpf::PfReq *rp = nullptr) {
  fl0 = fl1 = 0;
  if constexpr (FL) {
    fp.slot = fp.ev0 = fp.ev1 = fp.ev2 = fp.pf_rec = dpf::kNoSlot;
    fp.sens = false;
    fp.deferred = false;
  }
  if (!frame_ok(pin, buf_bytes)) {
    // layout contract violated: never touch memory outside the buffer
    o = out_record(pin.off, pin.len, DP_DONE_INTERNAL_FAILURE);
    if constexpr (MT) *pm = meta_none();
    return o.done;
  }
  TS_DECL
  Frame F;
  F.lds = slab;
  F.hs = hs;
  F.g = buf + pin.off;
  F.shift = (int)(pin.off & 15);
  F.len = pin.len;
  F.inwin = inwin;
  // the header window is staged in `slab` by the caller (kernel / dpemu_run)
  TS(0);
  Hdr H;
  if (!parse(F, 0, H)) {
    o = out_record(pin.off, pin.len, DP_DONE_NOT_ETHERNET);
    if constexpr (MT) *pm = meta_none();
    return o.done;
  }
  o.off = pin.off; o.len = pin.len;
  State S;
  S.done = DONE_NONE;
  S.flags = DP_META_INITIALIZED | DP_META_KEEP;
  S.has_vrf = false; S.vrf = 0; S.src_vni = 0; S.dst_vni = 0;
  S.has_oif = false; S.oif = 0; S.eg_code = DP_DONE_ROUTE_FAILURE; S.if_code = 255;
  S.eg_dmac = S.eg_smac = 0; S.fib = -1; S.vni_idx = -1; S.pair = -1;
  S.has_dscp = false; S.dscp = S.ecn = 0;
  S.fib_entry = 0xffffffffu; S.acl_rule = 0xffffffffu; S.acl = 0; S.nh_ref = NH_NONE;
  S.encap = false; S.o_eth = false; S.inner_l4_ck = false;
  S.ttl = 0; S.v4src = S.v4dst = 0;
  load_fields(F, H, S);
  TS(1);
  TRIP_ST(1);
  if (pin.flags & DP_IN_SEEDED_OVERLAY) {
    if (!enter_vni(g, S, pin.src_vni)) done(S, DP_DONE_UNROUTABLE);
  } else {
    stage_ingress(g, F, H, S, pin.iif);
    stage_ipforward(g, F, H, S);  // IP-Forward-1
  }
  TS(2);
  // IcmpErrorHandler (nat/src/icmp_handler/nf.rs:184-194): overlay ICMP error messages
  if (S.done == DONE_NONE && (S.flags & DP_META_IS_OVERLAY) && (H.l4 == L4_ICMP4 || H.l4 == L4_ICMP6) &&
      icmp_err_at(F, H.l4_off, H.l4 == L4_ICMP6)) {
    const uint8_t r = icmp_error_check(F, H, S);
    if (r != DONE_NONE) done(S, r);
    else if constexpr (FL) icmp_error_flow(*fc, F, H, S, fp);
  }
  // FlowLookup (flow-entry/src/flow_table/nf_lookup.rs:34-55); identity
  // without a flow table
  if constexpr (FL) {
    if (rp) {  // replay: the flow as FlowLookup attached it in the first pass
      if (rp->slot != dpf::kNoSlot) {
        fp.slot = rp->slot;
        fp.state = rp->state;
        fp.active = rp->status0 == DP_FLOW_ACTIVE;
        fp.fflags = rp->fflags0;
        fp.dst_vni = rp->dst_vni0;
        fp.related = rp->related0;
        fp.related_tag = rp->related_tag0;
        fp.genid = rp->genid0;
      }
    } else {
      dpf::FKey k;
      uint32_t st;
      if (S.done == DONE_NONE && (S.flags & DP_META_IS_OVERLAY) && !S.dst_vni && packet_fkey(F, H, S, k)) {
        uint4 v, w;
        const uint32_t sl = flow_probe(*fc, k, st, v, w);
        if (sl != dpf::kNoSlot) flow_attach(sl, st, v, w, fp);
      }
    }
  }
  TS(9);  // (the ICMP-error handler and FlowLookup)
  Pre P;
  TRIP_ST(2);
#ifndef DP_PROBE_NOFF
  stage_flow_filter<FL>(g, F, H, S, P, fp, fc, rp);
#else
  P.ffl = P.acl = P.nsrc = P.ndst = NO_PRE;
#endif
  TS(3);
  TRIP_ST(4);
#ifndef DP_PROBE_NOACL
  stage_acl<FL>(g, F, H, S, P, fp, fc, idx, rp);
#endif
  TS(4);
  TRIP_ST(5);
#ifndef DP_PROBE_NONAT
  stage_static_nat(g, F, H, S, P);
#endif
  if constexpr (SNAT) {
#ifndef DP_X_NOPF
    stage_portfw<FL>(F, H, S, fp, fc, idx, rp);
#endif
    stage_masquerade<FL>(F, H, S, fp, fc, idx, rp);
  }
#if !defined(DP_EMU) && defined(DP_EARLY_EFFECTS)
  // (A/B, measured slower: DESIGN §8) the packet's flow-table effects are all
  // decided here, so emitting them now, wave-aggregated over the lanes still
  // running, leaves the flow state dead through IP-Forward-2, Egress and
  // serialize
  if constexpr (FL) if (!rp) flow_effects<MT>(*fc, true, idx, fp);
#endif
  if constexpr (FL && SNAT) {
    if (fp.deferred) {  // finished by the replay pass
      o.done = DONE_NONE;
      return DONE_NONE;
    }
  }
  TS(5);
  TRIP_ST(6);
#ifndef DP_PROBE_NOIPF2
  stage_ipforward(g, F, H, S);  // IP-Forward-2
#endif
  TS(6);
  TRIP_ST(7);
  stage_egress(g, F, H, S);
  TS(7);
#ifdef DP_PROBE_NOSER
  if (false) {
#else
  if (S.done == DP_DONE_DELIVERED) {
#endif
    int st = serialize(F, H, S, fl0, fl1);
    S.flags &= ~DP_META_REFR_CHKSUM;
    if (S.done == DP_DONE_DELIVERED) {
      o.off = (uint32_t)((int)pin.off + st);
      o.len = (uint16_t)(F.len - st);
    }
  }
  o.done = S.done;
  o.meta_flags = (uint16_t)S.flags;
  o.oif = S.has_oif ? S.oif : 0;
  o.acl = S.acl;
  o.pad = 0;
  if constexpr (MT) {
    dp_pkt_meta_t m = meta_of(g, S);
    if constexpr (FL) if (fp.slot != dpf::kNoSlot) m.flow_ref = dpf::make_ref(fp.slot, fp.state);
    *pm = m;
  }
  TS(8);
  TS_FLUSH();
  return o.done;
}

#ifndef DP_EMU
// ---------------------------------------------------------------------------
// Kernel
// ---------------------------------------------------------------------------
// occupancy target: the compiler keeps VGPRs within 512 / DP_WAVES
#define DP_OCC __attribute__((amdgpu_waves_per_eu(DP_WAVES, DP_WAVES)))

// Wave-cooperative header-window staging and write-back.  M = the wave's
// largest chunk count rounded up to a power of two; in round r lane L moves
// chunk c of the wave's packet q, (q, c) = divmod(64 r + L, M): neighbouring
// lanes move neighbouring 16-byte chunks of one frame, so a wave-instruction
// touches 64 / M frames instead of 64.  Chunk c of packet q is window
// position 16 c of q's slab and buf + base_q + 16 c.
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int log2_up(int m) { return m <= 1 ? 0 : m <= 2 ? 1 : m <= 4 ? 2 : 3; }

__device__ __forceinline__ void wave_load_windows(const uint8_t *buf, uint8_t *slab_wave, uint32_t base, int nch) {
  const int lane = threadIdx.x & 63;
  const int lg = log2_up(wave_max(nch));
#pragma unroll 1
  for (int r = 0; r < (1 << lg); r++) {
    const int t = 64 * r + lane;
    const int q = t >> lg, c = t & ((1 << lg) - 1);
    const uint32_t qb = (uint32_t)__shfl((int)base, q);
    const int qn = __shfl(nch, q);
    if (c < qn) {
#ifdef DP_NT_LOADS  // A/B variant: the frames streamed in with the nontemporal policy
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(buf + qb + 16 * c));
      const uint4 v = make_uint4(t.x, t.y, t.z, t.w);
#else
      const uint4 v = *reinterpret_cast<const uint4 *>(buf + qb + 16 * c);
#endif
      lds_u32 *d = (lds_u32 *)(slab_wave + q * SLAB + 16 * c);
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  }
}

// 16-byte global store of the write-back and the out records.  DP_SC1_STORES
// (A/B variant): sc1 stores, which leave the XCD's L2 without keeping the
// line (MI355X_MICROARCH.md), so the streamed frames do not evict table lines.
__device__ __forceinline__ void st16(void *p, uint4 v) {
#if defined(DP_SC1_STORES)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(d) : "memory");
#elif defined(DP_NT_STORES)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4 *>(p));
#else
  *reinterpret_cast<uint4 *>(p) = v;
#endif
}

__device__ __forceinline__ void wave_store_windows(uint8_t *buf, const uint8_t *slab_wave, uint32_t base, int c0, int c1) {
  const int lane = threadIdx.x & 63;
  const int lg = log2_up(wave_max(c1));
#pragma unroll 1
  for (int r = 0; r < (1 << lg); r++) {
    const int t = 64 * r + lane;
    const int q = t >> lg, c = t & ((1 << lg) - 1);
    const uint32_t qb = (uint32_t)__shfl((int)base, q);
    const int q0 = __shfl(c0, q), q1 = __shfl(c1, q);
    if (c >= q0 && c < q1) {
      const lds_u32 *w = (const lds_u32 *)(slab_wave + q * SLAB + 16 * c);
      st16(buf + qb + 16 * c, make_uint4(w[0], w[1], w[2], w[3]));
    }
  }
}

// FL: the flows variant (a flow table is attached to the context); MT: meta
// records requested (meta != nullptr); RP: the replay pass of the packets
// that reached PortForwarder (FL only).
// VW: DP_V6W of the unit (a distinct kernel name per build of it).
template <bool FL, bool MT, bool RP, int VW>
__global__ void __launch_bounds__(TPB) DP_OCC
dp_pipeline_kernel(const uint8_t *__restrict__ img_base, const Image *__restrict__ im, uint8_t *__restrict__ buf,
                   uint64_t buf_bytes, const dp_pkt_in_t *__restrict__ in,
                   dp_pkt_out_t *__restrict__ out, dp_pkt_meta_t *__restrict__ meta, uint32_t n,
                   unsigned long long *__restrict__ part, dpf::FlowCtx fc) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_all[TPB * (SLAB + HS)];
#if DP_CTX
  // the context tables' copy, loaded beside the header windows (the one
  // barrier below covers both)
  __shared__ __attribute__((aligned(16))) uint8_t ctx_lds[DPD_CTX_MAX];
  {
    const uint32_t seg_lds[4] = {0u, im->ctx_pslots, im->ctx_prec, im->ctx_nh};
    const uint64_t seg_hbm[4] = {im->vni_slots, im->pairs.slots, im->pair_recs, im->nh_recs};
    const uint32_t seg_len[4] = {(im->vni_mask + 1) * (uint32_t)sizeof(VniRec),
                                 (im->pairs.mask + 1) * (uint32_t)sizeof(HashSlot),
                                 im->n_pair_recs * (uint32_t)sizeof(PairRec), im->n_nh * (uint32_t)sizeof(NhRec)};
#pragma unroll
    for (int q = 0; q < 4; q++)
      for (uint32_t u = threadIdx.x; u < seg_len[q] / 16; u += TPB)
        *reinterpret_cast<uint4 *>(ctx_lds + seg_lds[q] + 16 * u) =
            *reinterpret_cast<const uint4 *>(img_base + seg_hbm[q] + 16 * u);
  }
#endif
  uint8_t *slab_all = lds_all;
  uint8_t *hash_all = lds_all + TPB * SLAB;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  uint8_t *slab_wave = slab_all + (tid - lane) * SLAB;
  lds_u8 *slab = (lds_u8 *)(slab_all + tid * SLAB);
  // the replay pass (port forwarding, FL only): thread t finishes packet
  // pf_order[t] of the records dp_nat_prep ordered (fc.replay 1), of those
  // off the allocating lane (2: a masquerade split's, pf_cnt[12] 3 or 5 --
  // their decisions are dp_nat_resolve's or dp_nat_prep's, so this replay may
  // run beside the lane), of the steady refreshes dp_nat_prep resolved (4:
  // beside dp_nat_resolve and the lane) and then the rest off the lane (5),
  // or packet lane_order[t] (3: the lane's records, after it)
  constexpr bool rep = FL && RP;
  // chunk after chunk of TPB packets (DP_PERSIST), else the workgroup's one
#if DP_PERSIST
  for (uint32_t chunk = blockIdx.x; chunk * TPB < n; chunk += gridDim.x) {
#else
  {
  const uint32_t chunk = blockIdx.x;
#endif
  uint32_t i = chunk * TPB + tid;
  bool live = i < n;
  const dpf::PfReq *rp = nullptr;
  if constexpr (FL) {
    // the replay grid is the burst's; workgroups past the replayed packets
    // leave at once (uniform per workgroup: before any barrier)
    if constexpr (rep) {
      const bool split = fc.pf_cnt[12] == 3u || fc.pf_cnt[12] == 5u;
      const bool lanes = fc.replay == 3;
      const uint32_t cnt = !lanes ? fc.pf_cnt[1] : split ? fc.pf_cnt[11] : 0u;
      if (chunk * TPB >= cnt) return;
      live = i < cnt;
      i = live ? (lanes ? fc.lane_order[i] : fc.pf_order[i]) : n;
      if (live) rp = fc.pf + fc.pf_of[i];
      if (live && fc.replay != 1 && fc.replay != 3) {
        const uint32_t b = rp->bits;
        const bool keep = fc.replay == 4 ? (b & dpf::kPqSteady) != 0
                                         : !(fc.replay == 5 && (b & dpf::kPqSteady)) && !(split && (b & dpf::kPqLane));
        if (!keep) {
          live = false;
          i = n;
          rp = nullptr;
        }
      }
    }
  }
  dp_pkt_in_t pin{};
  if (live) pin = in[i];
  const uint32_t base = pin.off & ~15u;
  const int nch = live && frame_ok(pin, buf_bytes) ? window_chunks(pin) : 0;
  wave_load_windows(buf, slab_wave, base, nch);
  // wave-uniform: every live frame of the wave lies inside its window
  const bool all_fit = __ballot(live && ((pin.off & 15) + pin.len > (uint32_t)WIN || (pin.off & 1))) == 0;
  __syncthreads();
  uint8_t done_code = DONE_NONE;
  int fl0 = 0, fl1 = 0;
  FlowPk fp;
  fp.slot = dpf::kNoSlot;
  if (live) {
#if DP_CTX
    Img g{img_base, *im, (const lds_u8 *)ctx_lds};
#else
    Img g{img_base, *im};
#endif
    dp_pkt_out_t o;
    lds_u8 *hs = (lds_u8 *)(hash_all + tid * HS);
    dp_pkt_meta_t *pm = MT ? meta + i : nullptr;
    if (all_fit) done_code = process_packet<FL, MT>(g, slab, hs, buf, buf_bytes, pin, o, pm, fl0, fl1, true, &fc, fp, i, rp);
    else done_code = process_packet<FL, MT>(g, slab, hs, buf, buf_bytes, pin, o, pm, fl0, fl1, false, &fc, fp, i, rp);
    static_assert(sizeof(dp_pkt_out_t) == 16, "one 16-byte store");
    st16(out + i, *reinterpret_cast<const uint4 *>(&o));
  }
#ifndef DP_EARLY_EFFECTS  // the flow-table effects after the whole body, every lane of the wave
  if constexpr (FL) if (!rep) flow_effects<MT>(fc, live, i, fp);
#endif
  __syncthreads();
  // write-back: whole chunks by the wave, a partial tail by its owner
  wave_store_windows(buf, slab_wave, base, fl0 >> 4, fl1 >> 4);
  if (fl1 & 15) flush_range(buf + base, slab, fl1 & ~15, fl1);
  // DoneReason histogram: per wave by ballot, one atomic per reason present
  // into one of DPD_STAT_SLOTS partial histograms (dp_stats_reduce sums them)
  if (part) {
    unsigned long long pending = __ballot(live && done_code < DP_DONE_COUNT);
    const int slot = (int)((chunk * (TPB / 64) + (tid >> 6)) & (DPD_STAT_SLOTS - 1));
    while (pending) {
      const int leader = __ffsll(pending) - 1;
      const int r = __shfl((int)done_code, leader);
      const unsigned long long m = __ballot(live && (int)done_code == r) & pending;
      if (lane == leader) atomicAdd(&part[r * DPD_STAT_SLOTS + slot], (unsigned long long)__popcll(m));
      pending &= ~m;
    }
  }
  if (DP_PERSIST) __syncthreads();  // (the next chunk's windows reuse the slabs)
  }
}


// ---------------------------------------------------------------------------
// Port forwarding: the sequential pass (nat/src/portfw/nf.rs:326-397)
// ---------------------------------------------------------------------------
namespace pfw {

// PortFwTable::lookup_matching_rule -> LpmMap::lookup_cumulative
// (portfwtable/objects.rs:304-313, lpmmap.rs:108-116): the key's entries are
// sorted longest prefix first; the first that holds the address and whose
// range holds the port.  -1: none.
__device__ int32_t lookup(const Img &g, uint32_t src_vni, uint32_t proto, uint32_t fam, const uint32_t *a,
                          uint32_t port) {
  uint32_t v;
  if (!hash_find(g, g.im.pf_keys, src_vni, proto, 0, v)) return -1;
  const PfRuleRec *R = g.at<PfRuleRec>(g.im.pf_rules);
  for (uint32_t k = v >> 16, e = (v >> 16) + (v & 0xffffu); k < e; k++) {
    const PfRuleRec &r = R[k];
    if (r.fam != fam || port < r.ext_lo || port > r.ext_hi) continue;
    bool in = true;
    for (int j = 0; j < 4 && in; j++) {
      const int bits = (int)r.plen - 32 * j;
      const uint32_t m = bits >= 32 ? 0xffffffffu : bits <= 0 ? 0u : ~0u << (32 - bits);
      in = ((a[j] ^ r.ext[j]) & m) == 0;
    }
    if (in) return (int32_t)k;
  }
  return -1;
}
// Weak::upgrade of an entry: its index in these tables, -1 if gone
__device__ int32_t by_id(const Img &g, uint32_t id) {
  uint32_t v;
  return id && hash_find(g, g.im.pf_ids, id, 0, 0, v) ? (int32_t)v : -1;
}
__device__ bool unicast(uint32_t fam, const uint32_t *a) {  // UnicastIpv4Addr / UnicastIpv6Addr::new
  return fam == 4 ? !((a[0] >> 28) == 0xe || a[0] == 0xffffffffu) : (a[0] >> 24) != 0xff;
}
// PortFwEntry::map_address_port (objects.rs:168-203): the port's index in
// ext_ports into int_ports, the address's offset from the external network
// onto the internal one (wrapping), and a unicast result
__device__ bool map(const PfRuleRec &r, const uint32_t *a, uint32_t port, uint32_t *na, uint32_t &np) {
  if (port < r.ext_lo || port > r.ext_hi) return false;
  np = r.int_lo + (port - r.ext_lo);
  const int nw = r.fam == 4 ? 1 : 4;
  uint64_t borrow = 0, carry = 0;
  uint32_t off[4] = {0, 0, 0, 0};
  for (int j = nw - 1; j >= 0; j--) {
    const uint64_t d = (uint64_t)a[j] - r.ext[j] - borrow;
    off[j] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  for (int j = 3; j >= 0; j--) na[j] = 0;
  for (int j = nw - 1; j >= 0; j--) {
    const uint64_t v = (uint64_t)r.inn[j] + off[j] + carry;
    na[j] = (uint32_t)v;
    carry = v >> 32;
  }
  return unicast(r.fam, na);
}
// next_flow_status (portfw/protocol.rs:17-69)
__device__ uint32_t next_status(bool tcp, uint32_t fl, uint32_t act, uint32_t st) {
  if (tcp) {
    const bool fin = fl & 1, syn = fl & 2, rst = fl & 4, ack = fl & 16;
    if (act == DP_PF_DST_NAT) {
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
    return rst ? (uint32_t)DP_NFS_RESET : st;
  }
  if (act == DP_PF_DST_NAT) return st == DP_NFS_TWO_WAY ? (uint32_t)DP_NFS_ESTABLISHED : st;
  return st == DP_NFS_ONE_WAY ? (uint32_t)DP_NFS_TWO_WAY : st;
}

// The NAT pass's view of the table.  par: one of many lanes, each running the
// records of its own connections in packet order (dp_nat_resolve) -- the
// burst-wide counters (events, replaced fills, table length, probe bound) and
// the claim of a free slot are atomic; a connection's own slots are its lane's.
struct Seq {
  const dpf::FlowCtx &fc;
  const Img &g;
  bool par;
  // par: the lane's inserts, added to the table length once per wave when
  // the pass ends (no insert of a parallel pass reads the length: it cannot
  // reach the capacity)
  mutable uint32_t added = 0;
  // mode 4 (port forwarding near the capacity): the table length this
  // record's first insert meets, as the burst's earlier creations leave it
  // (dp_nat_admit_*: their new slots summed in packet order); kNoSlot: the
  // length as the table holds it
  mutable uint32_t adm = dpf::kNoSlot;
  __device__ uint32_t bump(uint32_t *c) const { return par ? atomicAdd(c, 1u) : (*c)++; }
  __device__ bool alive(uint32_t sl, uint32_t tag) const { return sl <= fc.mask && fc.slots[sl].state == tag; }
  // the pair is invalid for packet idx: either flow's burst-local mark says
  // so (invalidate_pair reaches the related flow only while it is alive)
  __device__ bool pair_valid(uint32_t sl, uint32_t idx) const {
    const dpf::FlowSlot &s = fc.slots[sl];
    if (s.mark <= idx) return false;
    return !(alive(s.related, s.related_tag) && fc.slots[s.related].mark <= idx);
  }
  // FlowInfo::invalidate_pair by packet idx: marks + the event apply turns
  // into the flows' status
  __device__ void invalidate(uint32_t sl, uint32_t idx) const {
    dpf::FlowSlot &s = fc.slots[sl];
    if (s.mark > idx + 1) s.mark = idx + 1;
    const uint32_t k = bump(&fc.events[0]);
    fc.events[1 + 2 * k] = sl;
    fc.events[2 + 2 * k] = s.state;
  }
  // the replaced fill's entry in the keyed index of replacements (dp_flow_fixup)
  __device__ void index_repl(uint32_t sl, uint32_t old, uint32_t r) const {
    uint32_t h = dpf::repl_hash(sl, old) & fc.rmask;
    const unsigned long long want = ((unsigned long long)fc.burst << 32) | sl;
    for (uint32_t p = 0; p <= fc.rmask;) {
      unsigned long long *w = reinterpret_cast<unsigned long long *>(&fc.repl[h].x);
      const unsigned long long cur = *w;
      if ((uint32_t)(cur >> 32) == fc.burst) {  // taken this burst: the next entry
        h = (h + 1) & fc.rmask;
        p++;
        continue;
      }
      if (atomicCAS(w, cur, want) != cur) continue;  // lost the race for it: look again
      fc.repl[h].z = old;
      fc.repl[h].w = r;
      return;
    }
  }
  __device__ void set_nfs(uint32_t sl, uint32_t st) const {
    dpf::FlowSlot &s = fc.slots[sl];
    s.pf = (s.pf & ~0xff00u) | (st << 8);
    if (alive(s.related, s.related_tag)) {
      dpf::FlowSlot &r = fc.slots[s.related];
      r.pf = (r.pf & ~0xff00u) | (st << 8);
    }
  }
  __device__ void reset_expiry(uint32_t sl, uint64_t dur) const {  // reset_expiry_unchecked (flow_info.rs:399-407)
    const uint64_t nw = fc.now + dur;
    if (nw >= fc.slots[sl].expires_at) fc.slots[sl].expires_at = nw;
  }
  // FlowTable::insert_common (flow-entry/src/flow_table/table.rs:215-260):
  // capacity (the second half of a pair is admitted at capacity while its
  // related flow is active), replacement of a flow of the same key (that
  // fill is Detached: gone from its slot), else the first free slot of the
  // key's probe sequence.  Returns the slot, kNoSlot when refused.
  __device__ uint32_t insert(const dpf::FKey &k, bool exception, uint32_t idx) const {
    uint64_t len = ((uint64_t)fc.tmeta[3] << 32) | fc.tmeta[2];
    if (par && adm != dpf::kNoSlot) len = (((uint64_t)fc.pf_cnt[7] << 32) | fc.pf_cnt[6]) + adm;
    if (len >= fc.capacity && !exception) return dpf::kNoSlot;
    const uint32_t home = dpf::fkey_hash(k) & fc.mask;
    const uint32_t bound = fc.tmeta[0];
    uint32_t i = home, found = dpf::kNoSlot, free_ = dpf::kNoSlot;
    for (uint32_t p = 0; p <= bound; p++, i = (i + 1) & fc.mask) {
      const dpf::FlowSlot &s = fc.slots[i];
      const uint32_t st = s.state & 3u;
      if (st == dpf::FS_EMPTY) { if (free_ == dpf::kNoSlot) free_ = i; break; }
      if (st == dpf::FS_TOMB) { if (free_ == dpf::kNoSlot) free_ = i; continue; }
      // a slot another lane is filling still shows the key of its last fill
      if (st == dpf::FS_BUSY) continue;
      if (s.src_vni == k.w[0] && s.fk == k.w[1] && s.ports == k.w[2] && s.src[0] == k.w[3] &&
          s.src[1] == k.w[4] && s.src[2] == k.w[5] && s.src[3] == k.w[6] && s.dst[0] == k.w[7] &&
          s.dst[1] == k.w[8] && s.dst[2] == k.w[9] && s.dst[3] == k.w[10]) { found = i; break; }
    }
    uint32_t sl = found;
    if (sl != dpf::kNoSlot) {
      // an invalidation of the replaced fill earlier in the burst reached its
      // related flow too (invalidate_pair): with the fill gone, that flow
      // carries the mark and the event itself
      const dpf::FlowSlot &x = fc.slots[sl];
      if (x.mark != dpf::kIdleMark && alive(x.related, x.related_tag)) {
        dpf::FlowSlot &y = fc.slots[x.related];
        if (y.mark > x.mark) y.mark = x.mark;
        const uint32_t e = bump(&fc.events[0]);
        fc.events[1 + 2 * e] = x.related;
        fc.events[2 + 2 * e] = y.state;
      }
      // the replaced fill, for the ACL verdicts that rest on it (dp_flow_fixup)
      const uint32_t r = bump(&fc.pf_cnt[2]);
      fc.pf_repl[4 * r] = sl;
      fc.pf_repl[4 * r + 1] = fc.slots[sl].state;
      fc.pf_repl[4 * r + 2] = idx;
      fc.pf_repl[4 * r + 3] = fc.slots[sl].mark;
      index_repl(sl, fc.slots[sl].state, r);
      // its FlowInfo is dropped when the burst ends, and with it the
      // allocation its masquerade state owns
      const dpf::FlowSlot &o = fc.slots[sl];
      if ((o.flags & dpf::kFlagMasq) && o.mq_rec && o.mq_gen == fc.mq_gen && fc.mq) {
        const uint32_t k = bump(&fc.pf_cnt[3]);
        fc.mq_rel[2 * k] = o.mq_rec - 1;
        fc.mq_rel[2 * k + 1] = o.pf >> 16;
      }
    } else if (!par) {
      if (len >= fc.hard) return dpf::kNoSlot;  // the table stays at most 7/8 full
      if (free_ == dpf::kNoSlot) {  // beyond the probe bound: the first free slot further on
        for (uint32_t p = bound + 1; p <= fc.mask; p++) {
          const uint32_t j = (home + p) & fc.mask;
          if ((fc.slots[j].state & 3u) != dpf::FS_FULL) { free_ = j; break; }
        }
        if (free_ == dpf::kNoSlot) return dpf::kNoSlot;
      }
      sl = free_;
      const uint32_t disp = (sl - home) & fc.mask;
      if (disp > fc.tmeta[0]) fc.tmeta[0] = disp;
      len++;
      fc.tmeta[2] = (uint32_t)len;
      fc.tmeta[3] = (uint32_t)(len >> 32);
    } else {
      // (the parallel pass runs only when no insert of the burst can meet the
      // capacity or the 7/8 bound: dp_nat_resolve)  The first free slot of
      // the probe sequence that this lane claims; other lanes claim theirs.
      sl = dpf::kNoSlot;
      for (uint32_t p = free_ == dpf::kNoSlot ? 0 : ((free_ - home) & fc.mask); p <= fc.mask; p++) {
        const uint32_t j = (home + p) & fc.mask;
        const uint32_t st = __hip_atomic_load(&fc.slots[j].state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((st & 3u) != dpf::FS_EMPTY && (st & 3u) != dpf::FS_TOMB) continue;
        if (atomicCAS(&fc.slots[j].state, st, (st & ~3u) | dpf::FS_BUSY) == st) { sl = j; break; }
      }
      if (sl == dpf::kNoSlot) return dpf::kNoSlot;
      // (the bound only grows: a displacement within the one read at this
      // insert's start needs nothing -- no agent-scope read of the one word
      // every lane's insert would otherwise queue on)
      const uint32_t disp = (sl - home) & fc.mask;
      if (disp > bound) atomicMax(&fc.tmeta[0], disp);
      added++;
    }
    dpf::FlowSlot &s = fc.slots[sl];
    const uint32_t old = s.state;  // (a claimed slot: BUSY, its tag kept)
    s.src_vni = k.w[0]; s.fk = k.w[1]; s.ports = k.w[2];
    for (int j = 0; j < 4; j++) { s.src[j] = k.w[3 + j]; s.dst[j] = k.w[7 + j]; }
    s.status = DP_FLOW_ACTIVE;
    s.related = dpf::kNoSlot;
    s.related_tag = 0;
    s.mark = dpf::kIdleMark;
    s.mq_rec = 0;
    s.state = ((((old >> 2) + 1) & 0x3fffffffu) << 2) | dpf::FS_FULL;
    return sl;
  }
};

__device__ inline uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// PortForwarder for one record, in packet order.
__device__ __forceinline__ void resolve_pf(const Seq &q, dpf::PfReq &R) {
  const dpf::FlowCtx &fc = q.fc;
  const Img &g = q.g;
  const uint32_t idx = R.idx;
  R.verdict = dpf::kPfForward;
  R.acl_over = 0;
  const bool attached = R.slot != dpf::kNoSlot;
  // the flow is still the fill FlowLookup attached (not replaced earlier in
  // the burst) and valid for this packet
  const bool same = attached && q.alive(R.slot, R.state);
  const bool valid = same && R.status0 == DP_FLOW_ACTIVE && q.pair_valid(R.slot, idx);
  // the ACL's "reply of a flow-scope-allowed flow" verdict needs the pair
  // still valid when the packet reached the ACL (dp_flow_fixup's rule)
  if (R.bits & dpf::kPqSens) {
    const bool rel = (R.bits & dpf::kPqRelated) && q.alive(R.related0, R.related_tag0);
    const bool ok = same && fc.slots[R.slot].mark > idx && (!rel || fc.slots[R.related0].mark > idx);
    if (!ok) {
      R.acl_over = R.acl_def;
      if (R.acl_def == 4) {  // the peering default denies: dropped at the ACL, its pair invalidated
        R.verdict = DP_DONE_ACL_DROPPED;
        if (same) q.invalidate(R.slot, idx);
        return;
      }
    }
  }
  if (!(R.bits & dpf::kPqPf)) return;
  const uint32_t fam = (R.proto >> 8) & 0xffu, proto = R.proto & 0xffu, tfl = R.proto >> 16;
  const bool tcp = R.bits & dpf::kPqTcp, ports = R.bits & (dpf::kPqTcp | dpf::kPqUdp);
  const uint32_t sport = R.ports >> 16, dport = R.ports & 0xffffu;
  // get_packet_port_fw_state (flow_state.rs:181-204): an Active flow with state
  if (valid && (fc.slots[R.slot].flags & dpf::kFlagPf)) {
    dpf::FlowSlot &f = fc.slots[R.slot];
    const uint32_t act = f.pf & 0xffu;
    int32_t e = by_id(g, f.pf_rule);
    if (e < 0) {
      // get_rule_from_pkt (nf.rs:206-324): would the current rules still do this?
      const PfRuleRec *RR = g.at<PfRuleRec>(g.im.pf_rules);
      uint32_t na[4], np;
      if (R.src_vni && ports) {
        if (act == DP_PF_DST_NAT) {
          const int32_t k = lookup(g, R.src_vni, proto, fam, R.dst, dport);
          if (k >= 0 && map(RR[k], R.dst, dport, na, np) && np == (f.pf >> 16) && RR[k].dst_vni == f.dst_vni &&
              na[0] == f.pf_ip[0] && na[1] == f.pf_ip[1] && na[2] == f.pf_ip[2] && na[3] == f.pf_ip[3])
            e = k;
        } else {
          const int32_t k = lookup(g, f.dst_vni, proto, f.pf_fam, f.pf_ip, f.pf >> 16);
          if (k >= 0 && map(RR[k], f.pf_ip, f.pf >> 16, na, np) && np == sport && RR[k].dst_vni == R.src_vni &&
              na[0] == R.src[0] && na[1] == R.src[1] && na[2] == R.src[2] && na[3] == R.src[3])
            e = k;
        }
      }
      if (e < 0) {
        R.verdict = DP_DONE_NAT_NOT_PORT_FORWARDED;
        q.invalidate(R.slot, idx);
        return;
      }
      // reassign_port_fw_rule, both flows (nf.rs:290-320)
      f.pf_rule = RR[e].id;
      if (q.alive(f.related, f.related_tag)) fc.slots[f.related].pf_rule = RR[e].id;
    }
    const PfRuleRec &E = g.at<PfRuleRec>(g.im.pf_rules)[e];
    R.nat = act | (f.pf & 0xffff0000u);
    for (int j = 0; j < 4; j++) R.nat_ip[j] = f.pf_ip[j];
    // refresh_port_fw_entry (flow_state.rs:216-264)
    const uint32_t cur = (f.pf >> 8) & 0xffu, nw = next_status(tcp, tfl, act, cur);
    q.set_nfs(R.slot, nw);
    if (nw == DP_NFS_CLOSED || nw == DP_NFS_RESET) { q.invalidate(R.slot, idx); return; }
    const uint64_t ext = nw == DP_NFS_ESTABLISHED ? E.estab_ns : E.init_ns;
    q.reset_expiry(R.slot, ext);
    if (nw == DP_NFS_ESTABLISHED && nw != cur && q.alive(f.related, f.related_tag)) q.reset_expiry(f.related, ext);
    f.genid = fc.genid;
    return;
  }
  // try_port_forwarding (nf.rs:174-204); can_be_port_forwarded (:54-94)
  if (!R.src_vni) { R.verdict = DP_DONE_INTERNAL_FAILURE; return; }
  const bool first_seg = (tfl & 2) && !(tfl & 0x3du);  // Tcp::is_first_segment (net/src/tcp/mod.rs:310-312)
  if (!(R.bits & dpf::kPqEth) || !ports || (tcp && !first_seg) || !unicast(fam, R.dst)) {
    R.verdict = DP_DONE_NAT_NOT_PORT_FORWARDED;
    return;
  }
  const int32_t e = lookup(g, R.src_vni, proto, fam, R.dst, dport);
  if (e < 0) { R.verdict = DP_DONE_NAT_NOT_PORT_FORWARDED; return; }
  const PfRuleRec &E = g.at<PfRuleRec>(g.im.pf_rules)[e];
  uint32_t na[4], np;
  if (!map(E, R.dst, dport, na, np)) { R.verdict = DP_DONE_INTERNAL_FAILURE; return; }
  // build_portfw_flow_keys (flow_state.rs:102-131): the key before static
  // NAT (or the current one) and the reverse of the DNATed current key
  dpf::FKey fk, rk;
  const uint32_t kind = tcp ? DP_FLOW_TCP : DP_FLOW_UDP;
  if (R.bits & dpf::kPqIkey) {
    for (int j = 0; j < 11; j++) fk.w[j] = R.ikey[j];
  } else {
    fk.w[0] = R.src_vni;
    fk.w[1] = fam | (kind << 8);
    fk.w[2] = R.ports;
    for (int j = 0; j < 4; j++) { fk.w[3 + j] = bswap(R.src[j]); fk.w[7 + j] = bswap(R.dst[j]); }
  }
  rk.w[0] = E.dst_vni;
  rk.w[1] = fam | (kind << 8);
  rk.w[2] = (np << 16) | sport;
  for (int j = 0; j < 4; j++) { rk.w[3 + j] = bswap(na[j]); rk.w[7 + j] = bswap(R.src[j]); }
  // (keys of distinct VPCs: related_pair never meets identical keys here)
  R.nat = DP_PF_DST_NAT | (np << 16);
  for (int j = 0; j < 4; j++) R.nat_ip[j] = na[j];
  const uint64_t exp = fc.now + E.init_ns;
  // compute_flow_flags_forward / _reverse (net/src/packet/meta.rs:264-287)
  const bool ss = R.bits & dpf::kPqSnatSrc, sd = R.bits & dpf::kPqSnatDst;
  const uint32_t fw_flags = DP_FLOW_INITIATOR | (ss ? DP_FLOW_REQ_STATIC_NAT_SRC : 0u) |
                            (sd ? DP_FLOW_REQ_STATIC_NAT_DST : 0u);
  const uint32_t rv_flags = (ss ? DP_FLOW_REQ_STATIC_NAT_DST : 0u) | (sd ? DP_FLOW_REQ_STATIC_NAT_SRC : 0u);
  const uint32_t sf = q.insert(fk, false, idx);
  if (sf == dpf::kNoSlot) { R.verdict = DP_DONE_FLOW_CAPACITY_EXCEEDED; return; }
  dpf::FlowSlot &F = fc.slots[sf];
  F.flags = fw_flags | dpf::kFlagPf;
  F.dst_vni = E.dst_vni;  // setup_forward_flow (flow_state.rs:133-157)
  F.genid = fc.genid;     // set_genid_pair
  F.expires_at = exp;
  F.pf = DP_PF_DST_NAT | (np << 16);  // NatFlowStatus::OneWay
  F.pf_rule = E.id;
  for (int j = 0; j < 4; j++) F.pf_ip[j] = na[j];
  F.pf_fam = fam;
  const uint32_t sr = q.insert(rk, true, idx);  // admitted at capacity: its related flow is Active
  if (sr == dpf::kNoSlot) {
    q.invalidate(sf, idx);
    R.verdict = DP_DONE_FLOW_CAPACITY_EXCEEDED;
    return;
  }
  dpf::FlowSlot &Rv = fc.slots[sr];
  Rv.flags = rv_flags | dpf::kFlagPf;
  Rv.dst_vni = E.src_vni;  // setup_reverse_flow (:159-177)
  Rv.genid = fc.genid;
  Rv.expires_at = exp;
  Rv.pf = DP_PF_SRC_NAT | (dport << 16);
  Rv.pf_rule = E.id;
  for (int j = 0; j < 4; j++) Rv.pf_ip[j] = R.dst[j];
  Rv.pf_fam = fam;
  F.related = sr;
  F.related_tag = Rv.state;
  Rv.related = sf;
  Rv.related_tag = F.state;
}

// ---------------------------------------------------------------------------
// Masquerade: the sequential pass (nat/src/masquerade/nf.rs:384-586)
// ---------------------------------------------------------------------------
constexpr uint64_t kMasqOneWayNs = 5000000000ull;   // MASQUERADE_ONEWAY_TIMEOUT (nf.rs:86)
constexpr uint64_t kMasqTwoWayNs = 3000000000ull;   // MASQUERADE_TWOWAY_TIMEOUT (:87)
constexpr uint64_t kMasqClosingNs = 2000000000ull;  // MASQUERADE_CLOSING_TIMEOUT (:88)

// next_flow_status (masquerade/protocol.rs:93-116) on the IP header's next
// header: UDP (a DstNat reply from port 53 / 853 / 8853 closes), ICMP, TCP by
// its flags -- port forwarding's machine with the initiator's side SrcNat
__device__ uint32_t masq_next_status(uint32_t proto, bool udp_hdr, uint32_t sport, uint32_t tfl, bool tcp_hdr,
                                     uint32_t act, uint32_t st) {
  const bool snat = act == DP_PF_SRC_NAT;
  if (proto == 17) {
    uint32_t n = st;
    if (snat) { if (st == DP_NFS_TWO_WAY) n = DP_NFS_ESTABLISHED; }
    else if (st == DP_NFS_ONE_WAY) n = DP_NFS_TWO_WAY;
    if (!snat && udp_hdr && (sport == 53 || sport == 853 || sport == 8853)) n = DP_NFS_CLOSED;
    return n;
  }
  if (proto == 1 || proto == 58) return (!snat && st == DP_NFS_ONE_WAY) ? (uint32_t)DP_NFS_TWO_WAY : st;
  if (proto == 6 && tcp_hdr) return next_status(true, tfl, snat ? DP_PF_DST_NAT : DP_PF_SRC_NAT, st);
  return st;
}

// From<&AllocatorError> for DoneReason (allocation.rs:59-73)
__device__ uint32_t masq_done(uint32_t e) {
  switch (e) {
    case dpm::NO_FREE_IP: case dpm::NO_PORT_BLOCK: case dpm::NO_FREE_PORT: return DP_DONE_NAT_OUT_OF_RESOURCES;
    case dpm::PORT_ALLOC_FAILED: case dpm::PORT_RESERVATION_FAILED: return DP_DONE_NAT_FAILURE;
    case dpm::INTERNAL: return DP_DONE_INTERNAL_FAILURE;
    default: return DP_DONE_FILTERED;  // Denied, NoPoolFound
  }
}

// The allocation path of Masquerade::masquerade_packet (nf.rs:384-475) in
// three parts, so the masquerading burst's allocating lane (dp_nat_lane) can
// serve a wave of records with one allocator step: masq_plan (what the record
// asks of the allocator, or its verdict without one), the allocation, masq_post
// (the checks between the allocation and the new pair, which give the tuple
// back) and masq_pair (the pair, create_flow_pair nf.rs:265-325).
struct MPlan {
  dpf::FKey ck, ik;       // the current key; the initial one (before static NAT)
  uint32_t kind, ikind, ifam, set, dport;
  bool allow_null;
  uint32_t sfail;         // a verdict masq_post gives whatever the tuple (0: none)
  bool eqp;               // the reverse key may equal the initial one (related_pair)
};

// A record of the allocating lane as dp_nat_lane_plan leaves it: 1 alone
// (live flow state decides it, or no room), 2 decided, 3 allocates
struct LanePlan {
  uint32_t rec, cls;
  MPlan m;
};
static_assert(sizeof(LanePlan) == 128, "one plan: eight 16-byte words");

// Is the record's flow valid for Masquerade with state (get_masquerade_state,
// nf.rs:198-213): the attached fill, Active for this packet (its own
// PortForwarder step included), holding masquerade state.
__device__ __forceinline__ bool masq_valid(const Seq &q, const dpf::PfReq &R) {
  const bool same = R.slot != dpf::kNoSlot && q.alive(R.slot, R.state);
  return same && R.status0 == DP_FLOW_ACTIVE && q.pair_valid(R.slot, R.idx + 1) &&
         (q.fc.slots[R.slot].flags & dpf::kFlagMasq);
}

// The record's current addresses and ports: PortForwarder's translation applied
__device__ __forceinline__ void masq_cur(const dpf::PfReq &R, uint32_t src[4], uint32_t dst[4], uint32_t &sport,
                                         uint32_t &dport) {
  const bool tcp = R.bits & dpf::kPqTcp, udp = R.bits & dpf::kPqUdp;
  sport = R.ports >> 16;
  dport = R.ports & 0xffffu;
  for (int j = 0; j < 4; j++) { src[j] = R.src[j]; dst[j] = R.dst[j]; }
  if ((R.bits & dpf::kPqPf) && (R.nat & 0xffu)) {
    const bool s = (R.nat & 0xffu) == DP_PF_SRC_NAT;
    for (int j = 0; j < 4; j++) (s ? src : dst)[j] = R.nat_ip[j];
    if (tcp || udp) (s ? sport : dport) = R.nat >> 16;
  }
}

// What the record asks of the allocator; false: it is decided without one
// (R.mverdict set).
__device__ __forceinline__ bool masq_plan(const dpf::FlowCtx &fc, dpf::PfReq &R, MPlan &m) {
  const uint32_t fam = (R.proto >> 8) & 0xffu, tfl = R.proto >> 16;
  const bool tcp = R.bits & dpf::kPqTcp, udp = R.bits & dpf::kPqUdp, icmp = R.bits & dpf::kPqIcmp;
  uint32_t src[4], dst[4], sport, dport;
  masq_cur(R, src, dst, sport, dport);
  dpm::View V{fc.mq};
  if (!fc.mq) { R.mverdict = DP_DONE_NAT_FAILURE; return false; }  // NoAllocator
  if (tcp && !((tfl & 2) && !(tfl & 0x3du))) { R.mverdict = DP_DONE_FILTERED; return false; }  // TCP without SYN
  // FlowKey::try_from(&Packet) (flow_key.rs:589-621): the current key
  if (tcp) m.kind = DP_FLOW_TCP;
  else if (udp) m.kind = DP_FLOW_UDP;
  else if (icmp) m.kind = (R.bits & dpf::kPqQuery) ? DP_FLOW_ICMP_QUERY : DP_FLOW_ICMP_OTHER;
  else { R.mverdict = DP_DONE_MALFORMED; return false; }  // FlowKeyError
  const uint32_t cports = m.kind == DP_FLOW_ICMP_OTHER ? 0u : ((sport << 16) | dport);
  m.ck.w[0] = R.src_vni;
  m.ck.w[1] = fam | (m.kind << 8);
  m.ck.w[2] = cports;
  for (int j = 0; j < 4; j++) { m.ck.w[3 + j] = bswap(src[j]); m.ck.w[7 + j] = bswap(dst[j]); }
  // the initial key: the one before static NAT, else the current one
  if (R.bits & dpf::kPqIkey) for (int j = 0; j < 11; j++) m.ik.w[j] = R.ikey[j];
  else m.ik = m.ck;
  m.ifam = m.ik.w[1] & 0xffu;
  m.ikind = m.ik.w[1] >> 8;
  m.dport = dport;
  const uint32_t iproto = m.ikind == DP_FLOW_TCP ? 6u : m.ikind == DP_FLOW_UDP ? 17u : m.ifam == 4 ? 1u : 58u;
  // NatAllocator::allocate (apalloc/mod.rs:317-375): the pool of (protocol,
  // VPCs, original source); a port, or an ICMP identifier (port 0 allowed)
  dpm::A128 sip{};
  if (m.ifam == 4) sip.w[3] = bswap(m.ik.w[3]);
  else for (int j = 0; j < 4; j++) sip.w[j] = bswap(m.ik.w[3 + j]);
  m.set = dpm::lookup(V, iproto | (m.ifam << 8), R.src_vni, R.dst_vni, sip);
  if (m.set == dpm::kNone) { R.mverdict = DP_DONE_FILTERED; return false; }  // Denied
  m.allow_null = iproto == 1 || iproto == 58;
  // masq_post's verdicts that do not rest on the tuple
  m.sfail = m.kind == DP_FLOW_ICMP_OTHER ? (uint32_t)DP_DONE_NAT_FAILURE  // UnexpectedKeyVariant
          : (m.ikind != DP_FLOW_TCP && m.ikind != DP_FLOW_UDP && m.ikind != DP_FLOW_ICMP_QUERY)
              ? (uint32_t)DP_DONE_NAT_FAILURE  // IcmpUnsupportedCategory
              : 0u;
  // related_pair's equal keys need the reverse key's source (the current
  // destination) to be the initial source, in the destination VPC
  bool eq = m.ik.w[0] == R.dst_vni && m.ik.w[1] == m.ck.w[1];
  for (int j = 0; j < 4; j++) eq = eq && m.ik.w[3 + j] == m.ck.w[7 + j];
  m.eqp = eq;
  return true;
}

// The reverse of the current key towards the allocated tuple
// (new_reverse_session, nf.rs:327-373)
__device__ __forceinline__ void masq_rk(const dpf::PfReq &R, const MPlan &m, const uint32_t aip[4], uint32_t aport,
                                        dpf::FKey &rk) {
  rk.w[0] = R.dst_vni;
  rk.w[1] = m.ck.w[1];
  for (int j = 0; j < 4; j++) { rk.w[3 + j] = m.ck.w[7 + j]; rk.w[7 + j] = bswap(aip[j]); }
  rk.w[2] = m.kind == DP_FLOW_ICMP_QUERY ? aport << 16 : (m.dport << 16) | aport;
}

// The checks between the allocation and the pair: a verdict that gives the
// tuple back, or 0.
__device__ __forceinline__ uint32_t masq_post(const dpf::PfReq &R, const MPlan &m, const uint32_t aip[4],
                                              uint32_t aport) {
  const uint32_t fam = (R.proto >> 8) & 0xffu;
  if (!unicast(fam, aip)) return DP_DONE_FILTERED;
  if (m.kind == DP_FLOW_TCP || m.kind == DP_FLOW_UDP) {
    if (aport == 0) return DP_DONE_MALFORMED;  // InvalidPort
  } else if (m.kind != DP_FLOW_ICMP_QUERY) {
    return DP_DONE_NAT_FAILURE;  // UnexpectedKeyVariant
  }
  // get_reverse_mapping: the original source tuple
  if (m.ikind != DP_FLOW_TCP && m.ikind != DP_FLOW_UDP && m.ikind != DP_FLOW_ICMP_QUERY)
    return DP_DONE_NAT_FAILURE;  // IcmpUnsupportedCategory
  dpf::FKey rk;
  masq_rk(R, m, aip, aport, rk);
  bool eq = true;
  for (int j = 0; j < 11; j++) eq = eq && m.ik.w[j] == rk.w[j];
  return eq ? (uint32_t)DP_DONE_INTERNAL_FAILURE : 0u;  // related_pair
}

__device__ __forceinline__ void masq_aip(const dpf::FlowCtx &fc, const dpf::PfReq &R, uint32_t rec, uint32_t aip[4]) {
  const dpm::View V{fc.mq};
  const dpm::A128 aa = dpm::addr_of(V, V.recs()[rec]);
  const uint32_t fam = (R.proto >> 8) & 0xffu;
  for (int j = 0; j < 4; j++) aip[j] = 0;  // big-endian words, v4 in word 0
  if (fam == 4) aip[0] = aa.w[3];
  else for (int j = 0; j < 4; j++) aip[j] = aa.w[j];
}

// create_flow_pair (nf.rs:265-325) for an allocation that passed masq_post.
// false: refused at capacity (the allocation is the caller's to give back
// when the forward flow was refused; R.mverdict set).
__device__ __forceinline__ bool masq_pair(const Seq &q, dpf::PfReq &R, const MPlan &m, uint32_t rec,
                                          uint32_t aport, const uint32_t aip[4], bool &give_back) {
  const dpf::FlowCtx &fc = q.fc;
  const uint32_t idx = R.idx;
  const uint32_t fam = (R.proto >> 8) & 0xffu;
  dpf::FKey rk;
  masq_rk(R, m, aip, aport, rk);
  const uint32_t rport = m.ik.w[2] >> 16;
  const bool rident = m.ikind == DP_FLOW_ICMP_QUERY;
  const bool ss = R.bits & dpf::kPqSnatSrc, sd = R.bits & dpf::kPqSnatDst;
  const uint32_t fw_flags = DP_FLOW_INITIATOR | (ss ? DP_FLOW_REQ_STATIC_NAT_SRC : 0u) |
                            (sd ? DP_FLOW_REQ_STATIC_NAT_DST : 0u);
  const uint32_t rv_flags = (ss ? DP_FLOW_REQ_STATIC_NAT_DST : 0u) | (sd ? DP_FLOW_REQ_STATIC_NAT_SRC : 0u);
  const dpm::View V{fc.mq};
  const int64_t genid = V.h().genid;  // set_genid_pair(allocator.genid())
  const uint64_t exp = fc.now + kMasqOneWayNs;
  const uint32_t idle_s = (uint32_t)(V.sets()[m.set].idle_ns / 1000000000ull);
  give_back = false;
  const uint32_t sf = q.insert(m.ik, false, idx);
  if (sf == dpf::kNoSlot) {  // the allocation drops here
    give_back = true;
    R.mverdict = DP_DONE_FLOW_CAPACITY_EXCEEDED;
    return false;
  }
  dpf::FlowSlot &F = fc.slots[sf];
  F.flags = fw_flags | dpf::kFlagMasq | (m.allow_null ? dpf::kFlagMasqIdent : 0u);
  F.dst_vni = R.dst_vni;  // setup_flow_masquerade_state: the forward flow to dst_vpcd
  F.genid = genid;
  F.expires_at = exp;
  F.pf = DP_PF_SRC_NAT | (aport << 16);  // NatFlowStatus::OneWay
  F.pf_rule = idle_s;
  for (int j = 0; j < 4; j++) F.pf_ip[j] = aip[j];
  F.pf_fam = fam;
  F.mq_rec = rec + 1;
  F.mq_gen = fc.mq_gen;
  const uint32_t sr = q.insert(rk, true, idx);  // admitted at capacity: its related flow is Active
  if (sr == dpf::kNoSlot) {
    q.invalidate(sf, idx);
    R.mverdict = DP_DONE_FLOW_CAPACITY_EXCEEDED;
    return false;
  }
  dpf::FlowSlot &Rv = fc.slots[sr];
  Rv.flags = rv_flags | dpf::kFlagMasq | (rident ? dpf::kFlagMasqIdent : 0u);
  Rv.dst_vni = R.src_vni;  // the reverse one to src_vpcd
  Rv.genid = genid;
  Rv.expires_at = exp;
  Rv.pf = DP_PF_DST_NAT | (rport << 16);
  Rv.pf_rule = idle_s;
  for (int j = 0; j < 4; j++) Rv.pf_ip[j] = 0;
  if (m.ifam == 4) Rv.pf_ip[0] = bswap(m.ik.w[3]);
  else for (int j = 0; j < 4; j++) Rv.pf_ip[j] = bswap(m.ik.w[3 + j]);
  Rv.pf_fam = m.ifam;
  F.related = sr;
  F.related_tag = Rv.state;
  Rv.related = sf;
  Rv.related_tag = F.state;
  // the packet with the forward state (no Ethernet header: a failure that
  // invalidates the new pair -- never here, every frame has one)
  R.mnat = DP_PF_SRC_NAT | (m.allow_null ? 0x100u : 0u) | (aport << 16);
  for (int j = 0; j < 4; j++) R.mnat_ip[j] = aip[j];
  return true;
}

// Masquerade::masquerade_packet (nf.rs:384-475) for one record, after its
// PortForwarder decision (the packet as PortForwarder left it).
__device__ __forceinline__ void resolve_masq(const Seq &q, dpf::PfReq &R) {
  const dpf::FlowCtx &fc = q.fc;
  const uint32_t idx = R.idx;
  const uint32_t fam = (R.proto >> 8) & 0xffu, proto = R.proto & 0xffu, tfl = R.proto >> 16;
  const bool tcp = R.bits & dpf::kPqTcp, udp = R.bits & dpf::kPqUdp, icmp = R.bits & dpf::kPqIcmp;
  // get_masquerade_state (nf.rs:198-213): the attached flow, still that fill,
  // Active for this packet (its own PortForwarder step included), with state
  if (masq_valid(q, R)) {
    uint32_t src[4], dst[4], sport, dport;
    masq_cur(R, src, dst, sport, dport);
    dpf::FlowSlot &f = fc.slots[R.slot];
    const uint32_t act = f.pf & 0xffu, port = f.pf >> 16;
    const bool ident = f.flags & dpf::kFlagMasqIdent;
    // refresh_masquerade_state (nf.rs:151-194)
    const uint32_t cur = (f.pf >> 8) & 0xffu;
    const uint32_t nw = masq_next_status(proto, udp, sport, tfl, tcp, act, cur);
    q.set_nfs(R.slot, nw);
    if (nw == DP_NFS_CLOSED || nw == DP_NFS_RESET) {
      q.invalidate(R.slot, idx);  // and the packet is still translated
    } else if (nw != DP_NFS_ONE_WAY) {
      const uint64_t ext = nw == DP_NFS_TWO_WAY ? kMasqTwoWayNs
                         : nw == DP_NFS_ESTABLISHED ? (uint64_t)f.pf_rule * 1000000000ull : kMasqClosingNs;
      q.reset_expiry(R.slot, ext);
      if (nw == DP_NFS_ESTABLISHED && nw != cur && q.alive(f.related, f.related_tag)) q.reset_expiry(f.related, ext);
    }
    // masquerade (packet.rs:35-195): a SrcNat state needs a unicast address, the
    // packet one of the state's family and a TCP / UDP / ICMP header
    if ((act == DP_PF_SRC_NAT && !unicast(f.pf_fam, f.pf_ip)) || f.pf_fam != fam || !(tcp || udp || icmp)) {
      R.mverdict = DP_DONE_NAT_FAILURE;
      return;
    }
    R.mnat = act | (ident ? 0x100u : 0u) | (port << 16);
    for (int j = 0; j < 4; j++) R.mnat_ip[j] = f.pf_ip[j];
    return;
  }
  MPlan m;
  if (!masq_plan(fc, R, m)) return;
  const dpm::View V{fc.mq};
  uint32_t rec = 0, aport = 0;
  const uint32_t e = dpm::set_alloc(V, m.set, m.allow_null, rec, aport);
  if (e != dpm::OK) { R.mverdict = masq_done(e); return; }
  uint32_t aip[4];
  masq_aip(fc, R, rec, aip);
  const uint32_t v = masq_post(R, m, aip, aport);
  if (v) { dpm::release(V, rec, aport); R.mverdict = v; return; }
  bool give_back;
  if (!masq_pair(q, R, m, rec, aport, aip, give_back) && give_back) dpm::release(V, rec, aport);
}

// One record, in packet order: PortForwarder, then Masquerade on what it left.
__device__ __forceinline__ void resolve_one(const Seq &q, dpf::PfReq &R) {
  R.mverdict = dpf::kPfForward;
  resolve_pf(q, R);
  if ((R.bits & dpf::kPqMasq) && R.verdict == dpf::kPfForward) resolve_masq(q, R);
}

// ---------------------------------------------------------------------------
// The NAT pass in parallel: connections
// ---------------------------------------------------------------------------
// PortForwarder's decisions couple only the records of one connection (its
// flow pair, the pair a packet of it creates) and the table-wide insert
// admission.  A record's connection is named by the key its reply direction
// carries: the reverse flow's key (a forward flow's related flow, or derived
// from its state), or, for a packet that may create a pair, the reverse key
// try_port_forwarding would insert (nf.rs:174-204, flow_state.rs:102-131).
// Records of one connection run in packet order on one lane; connections run
// in parallel.  Hash collisions only merge connections.

// The reverse key the creation path would insert for this record (the same
// preconditions and mapping as resolve_pf's creation), false: it creates none.
__device__ bool creation_rk(const Img &g, const dpf::PfReq &R, dpf::FKey &rk) {
  if (!(R.bits & dpf::kPqPf) || !R.src_vni) return false;
  const uint32_t fam = (R.proto >> 8) & 0xffu, proto = R.proto & 0xffu, tfl = R.proto >> 16;
  const bool tcp = R.bits & dpf::kPqTcp, ports = R.bits & (dpf::kPqTcp | dpf::kPqUdp);
  const bool first_seg = (tfl & 2) && !(tfl & 0x3du);
  if (!(R.bits & dpf::kPqEth) || !ports || (tcp && !first_seg) || !unicast(fam, R.dst)) return false;
  const uint32_t sport = R.ports >> 16, dport = R.ports & 0xffffu;
  // the address copied first: lookup / map index it with loop bounds the
  // family sets, which would otherwise keep the whole record in scratch
  uint32_t dst[4];
#pragma unroll
  for (int j = 0; j < 4; j++) dst[j] = R.dst[j];
  const int32_t e = lookup(g, R.src_vni, proto, fam, dst, dport);
  if (e < 0) return false;
  const PfRuleRec &E = g.at<PfRuleRec>(g.im.pf_rules)[e];
  uint32_t na[4], np;
  if (!map(E, dst, dport, na, np)) return false;
  rk.w[0] = E.dst_vni;
  rk.w[1] = fam | ((tcp ? DP_FLOW_TCP : DP_FLOW_UDP) << 8);
  rk.w[2] = (np << 16) | sport;
  for (int j = 0; j < 4; j++) { rk.w[3 + j] = bswap(na[j]); rk.w[7 + j] = bswap(R.src[j]); }
  return true;
}

__device__ inline dpf::FKey slot_key(const dpf::FlowSlot &s) {
  dpf::FKey k;
  k.w[0] = s.src_vni; k.w[1] = s.fk; k.w[2] = s.ports;
  for (int j = 0; j < 4; j++) { k.w[3 + j] = s.src[j]; k.w[7 + j] = s.dst[j]; }
  return k;
}

// A burst with both kinds of record (mode 5): port forwarding's connections
// run as connection lanes beside the masquerade split's (dp_nat_resolve),
// before the allocating lane (dp_nat_lane).  That is the one-lane pass's
// outcome when no port-forwarding connection meets a masquerade record's
// flows and the inserts cannot meet the capacity (room for every pair):
//  - a port-forwarding record on a masqueraded flow (its creation would
//    replace it) or a creation whose reverse key another flow holds: no
//    connection key (conn_key), the burst runs on one lane (pf_cnt[5]);
//  - a masquerading record on a port-forwarded flow (its allocation would
//    replace that flow), a record that both forwards and masquerades: one
//    lane (dp_nat_mark, pf_cnt[30]);
//  - a masquerading record without a live flow whose initial key is the
//    reverse key a creation of the burst inserts (the forwarded host's first
//    packet back in the same burst, before FlowLookup could see the new pair):
//    one lane (dp_nat_prep registers the creations' reverse keys, dp_nat_cross
//    looks the initial keys up, pf_cnt[30]);
//  - a masquerade allocation never hands out a forwarded public tuple of its
//    manifest (the claims, apalloc/setup.rs:73-91), so no pair the lane
//    creates meets a key a creation inserts.
// A record's initial key cannot be a creation's forward key: the same key
// from the same VPC gets the same flow-filter decision, so the same kind.
// Port-forwarding connection keys carry bit 31, masquerade ones (a slot
// index) never do, so the two kinds never share a connection.
[[maybe_unused]] constexpr uint32_t kPfConnBit = 0x80000000u;

// The key a masquerading record's allocation inserts first (masq_plan's
// initial key) when it has no port forwarding; false: it inserts none.
__device__ bool masq_ik(const dpf::PfReq &R, dpf::FKey &k) {
  if (R.bits & dpf::kPqIkey) {
    for (int j = 0; j < 11; j++) k.w[j] = R.ikey[j];
    return true;
  }
  const uint32_t fam = (R.proto >> 8) & 0xffu;
  uint32_t kind;
  if (R.bits & dpf::kPqTcp) kind = DP_FLOW_TCP;
  else if (R.bits & dpf::kPqUdp) kind = DP_FLOW_UDP;
  else if (R.bits & dpf::kPqIcmp) kind = (R.bits & dpf::kPqQuery) ? DP_FLOW_ICMP_QUERY : DP_FLOW_ICMP_OTHER;
  else return false;
  k.w[0] = R.src_vni;
  k.w[1] = fam | (kind << 8);
  k.w[2] = kind == DP_FLOW_ICMP_OTHER ? 0u : R.ports;
  for (int j = 0; j < 4; j++) { k.w[3 + j] = bswap(R.src[j]); k.w[7 + j] = bswap(R.dst[j]); }
  return true;
}

// The creations' reverse keys of a mixed burst, in dup_tab under the tag
// ~burst (dp_nat_lane_plan later claims entries under the tag burst and takes
// these for empty ones): the slot from one hash of the key, the tag word from
// another, as dp_nat_lane_plan keys its entries.
__device__ __forceinline__ void cross_hash(const dpf::FlowCtx &fc, const dpf::FKey &k, uint32_t &x,
                                           unsigned long long &want) {
  x = dpm::kmix(dpf::fkey_hash(k), 0x5bd1e995u, 0u) & fc.grp_mask;
  const uint32_t h2 = dpm::kmix(dpm::kmix(k.w[0], k.w[1], k.w[2]), dpm::kmix(k.w[3], k.w[4], k.w[5]) ^ k.w[6],
                                dpm::kmix(k.w[7], k.w[8], k.w[9]) ^ k.w[10]);
  want = ((unsigned long long)~fc.burst << 32) | h2;
}
// false: the table is full (the caller sends the burst to one lane)
__device__ bool cross_put(const dpf::FlowCtx &fc, const dpf::FKey &k) {
  uint32_t x;
  unsigned long long want;
  cross_hash(fc, k, x, want);
  for (uint32_t p = 0; p <= fc.grp_mask; p++, x = (x + 1) & fc.grp_mask) {
    const unsigned long long cur = __hip_atomic_load(&fc.dup_tab[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == want) return true;
    if ((uint32_t)(cur >> 32) == ~fc.burst) continue;
    const unsigned long long got = atomicCAS(&fc.dup_tab[x], cur, want);
    if (got == cur || got == want) return true;
  }
  return false;
}
// may `k` be a registered reverse key (hash equality; a full table: yes)
__device__ bool cross_has(const dpf::FlowCtx &fc, const dpf::FKey &k) {
  uint32_t x;
  unsigned long long want;
  cross_hash(fc, k, x, want);
  for (uint32_t p = 0; p <= fc.grp_mask; p++, x = (x + 1) & fc.grp_mask) {
    const unsigned long long cur = __hip_atomic_load(&fc.dup_tab[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == want) return true;
    if ((uint32_t)(cur >> 32) != ~fc.burst) return false;
  }
  return true;
}

// The record's connection key; false: the record needs the sequential pass
// (masquerade: one allocator; a flow without port-forwarding state; a pair it
// may create that is not its flow's).
// cross: a mixed burst (mode 5): a creation's reverse key is registered for
// dp_nat_cross (cross_put; a full table refuses the record).
__device__ bool conn_key(const Img &g, const dpf::FlowCtx &fc, const dpf::PfReq &R, uint32_t &key,
                         bool cross = false) {
  if (R.bits & dpf::kPqMasq) return false;
  dpf::FKey rk;
  const bool cand = creation_rk(g, R, rk);
  if (cand) {
    // a flow already holding that key must be a port-forwarded reply flow
    // (whose packets name the same connection); anything else couples
    // connections
    uint32_t st;
    uint4 v, w;
    const uint32_t z = flow_probe(fc, rk, st, v, w);
    if (z != dpf::kNoSlot && !((v.y & dpf::kFlagPf) && (fc.slots[z].pf & 0xffu) == DP_PF_SRC_NAT)) return false;
  }
  if (R.slot == dpf::kNoSlot) {
    if (cand && cross) {
      if (!cross_put(fc, rk)) return false;
      atomicAdd(&fc.pf_cnt[32], 1u);
    }
    key = cand ? dpf::fkey_hash(rk) : (R.idx * 0x9E3779B1u) ^ 0x5bd1e995u;  // no flow, no pair: alone
    return true;
  }
  const dpf::FlowSlot &A = fc.slots[R.slot];
  if (!(A.flags & dpf::kFlagPf)) return false;
  dpf::FKey ak;
  if ((A.pf & 0xffu) == DP_PF_SRC_NAT) {
    ak = slot_key(A);  // the reverse flow itself
  } else if (A.related <= fc.mask && fc.slots[A.related].state == A.related_tag) {
    ak = slot_key(fc.slots[A.related]);
  } else {  // the reverse key from the forward flow's state
    ak.w[0] = A.dst_vni;
    ak.w[1] = A.fk;
    ak.w[2] = (A.pf & 0xffff0000u) | (A.ports >> 16);
    for (int j = 0; j < 4; j++) { ak.w[3 + j] = bswap(A.pf_ip[j]); ak.w[7 + j] = A.src[j]; }
  }
  if (cand)
    for (int j = 0; j < 11; j++)
      if (rk.w[j] != ak.w[j]) return false;
  if (cand && cross) {
    if (!cross_put(fc, rk)) return false;
    atomicAdd(&fc.pf_cnt[32], 1u);
  }
  key = dpf::fkey_hash(ak);
  return true;
}

// The records of one connection (a list through grp_next, pushed in any
// order) sorted by packet index: a merge sort of the linked list.
// (The links are read and rewritten through relaxed atomics: a lane's
// rewrite of a link must be what its next read of that link returns -- with
// plain accesses the GPU build lost records of longer lists.)
__device__ inline unsigned long long link_ld(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void link_st(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ uint32_t sort_conn(unsigned long long *nx, uint32_t list) {
  auto next = [&](uint32_t r) { return (uint32_t)link_ld(&nx[r]); };
  auto set_next = [&](uint32_t r, uint32_t v) { link_st(&nx[r], (link_ld(&nx[r]) & 0xffffffff00000000ull) | v); };
  if (list == dpf::kNoSlot || next(list) == dpf::kNoSlot) return list;
  for (uint32_t insize = 1;; insize *= 2) {
    uint32_t p = list, tail = dpf::kNoSlot, merges = 0;
    list = dpf::kNoSlot;
    while (p != dpf::kNoSlot) {
      merges++;
      uint32_t q = p, psize = 0;
      for (uint32_t i = 0; i < insize; i++) {
        psize++;
        q = next(q);
        if (q == dpf::kNoSlot) break;
      }
      uint32_t qsize = insize;
      while (psize > 0 || (qsize > 0 && q != dpf::kNoSlot)) {
        uint32_t e;
        if (psize == 0) { e = q; q = next(q); qsize--; }
        else if (qsize == 0 || q == dpf::kNoSlot || (link_ld(&nx[p]) >> 32) <= (link_ld(&nx[q]) >> 32)) {
          e = p; p = next(p); psize--;
        }
        else { e = q; q = next(q); qsize--; }
        if (tail != dpf::kNoSlot) set_next(tail, e);
        else list = e;
        tail = e;
      }
      p = q;
    }
    set_next(tail, dpf::kNoSlot);
    if (merges <= 1) return list;
  }
}

// ---------------------------------------------------------------------------
// The masquerading burst, split (dp_nat_prep, dp_nat_resolve, dp_nat_lane)
// ---------------------------------------------------------------------------
// Masquerade couples a burst's records through one allocator only where a
// record allocates, and the flows a record reads are its own connection's
// except where an allocation's new pair replaces them.  So a masquerading
// burst is run in two parts whose outcome is the one-lane pass's in packet
// order:
//  - connection lanes (dp_nat_resolve): the records attached to one flow pair
//    that holds masquerade state with a live allocation, in packet order --
//    refreshes of NatFlowStatus and expiry, closes and resets, the ACL's flow
//    verdicts -- up to the first record that would allocate (its flow no
//    longer valid); that record and the rest of the connection go to
//  - the allocating lane (dp_nat_lane): every other masquerading record, in
//    packet order: first packets, packets on flows without (valid) state,
//    what the connection lanes left.  Its records are taken 64 at a time;
//    runs of records that allocate are served by one allocator step for the
//    whole wave (the k-th of them takes the k-th free port of the address's
//    thread block, as one after the other would) and create their pairs in
//    parallel; a record whose outcome rests on live flow state runs alone.
// Why the parts commute: a connection lane's pair keeps its tuple allocated
// for the whole burst (the forward flow owns it; a replaced fill gives it
// back only when the burst ends), so no allocation of the burst hands it out
// again, and a record whose initial key is the pair's key is attached to the
// pair (FlowLookup found it) and so runs in the connection's order.  What
// would break that is refused at dp_nat_prep: a port-forwarding record in the
// burst, or a masquerading packet whose own peer could masquerade towards a
// public address (masq_back: a reverse key allocated this burst could then be
// another record's initial key); those bursts run on one lane.  The table's
// capacity and 7/8 bound concern the allocating lane alone (the connection
// lanes insert nothing): without room for every pair it could create, it
// takes its records one by one.

// The NAT pass's mode for this burst: 1 one lane in packet order, 2
// connections in parallel (port forwarding: when no insert of the burst can
// meet the capacity or the 7/8 bound), 3 split (masquerade: only the
// allocating lane inserts, and it takes its records one by one in packet
// order when room is short -- dp_nat_lane), 4 connections in parallel with
// insert_common's capacity admissions decided beforehand in packet order
// (port forwarding without room for every pair: dp_nat_admit_*), 5 mixed:
// port-forwarding connections in parallel beside the masquerade split (a
// burst holding both kinds of record, with room for every pair; below).  pre:
// the mode before dp_nat_admit_plan has looked at the connections (4 may turn
// 1); dp_nat_prep and dp_nat_cross may still turn 5 into 1.
__device__ __forceinline__ uint32_t nat_mode(const dpf::FlowCtx &fc, bool pre = false) {
  if (fc.force_seq == 1 || fc.pf_cnt[5]) return 1u;
  const uint64_t len0 = ((uint64_t)fc.pf_cnt[7] << 32) | fc.pf_cnt[6];
  const uint64_t total = fc.pf_cnt[1];
  const bool room = len0 + 2ull * total <= fc.capacity && len0 + 2ull * total <= fc.hard;
  if (fc.pf_cnt[8]) {
    if (fc.pf_cnt[10] || !fc.lane_plan) return 1u;
    if (!fc.pf_cnt[9]) return 3u;
    // (mixed: room for every slot the burst may add, pf_cnt[31] as dp_nat_prep
    // bounds it -- before it has, the mode prep runs in)
    const uint64_t add = fc.pf_cnt[31];
    const bool mroom = len0 + add <= fc.capacity && len0 + add <= fc.hard;
    return mroom && !fc.pf_cnt[30] && fc.force_seq != 4 ? 5u : 1u;
  }
  if (room) return 2u;
  // (the 7/8 bound out of reach: only the capacity can refuse, and only a
  // creation's first insert)
  if (fc.force_seq != 3 && len0 + 2ull * total <= fc.hard && fc.capacity <= fc.hard && total <= (4u << 20) &&
      (pre || !fc.pf_cnt[17]))
    return 4u;
  return 1u;
}

// the modes that run the masquerade split (connection lanes, the allocating lane)
__device__ __forceinline__ bool split_mode(uint32_t m) { return m == 3u || m == 5u; }

__device__ __forceinline__ void flag_once(uint32_t *w) {
  if (!__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicOr(w, 1u);
}
// flag_once for the wave: one lane of those that want it (a chip's worth of
// lanes reading one word would queue at its L2 channel)
__device__ __forceinline__ void flag_wave(uint32_t *w, bool want) {
#ifdef DP_EMU
  if (want) flag_once(w);
#else
  const uint64_t m = __ballot(want);
  if (m && (int)(threadIdx.x & 63) == __ffsll((long long)m) - 1) flag_once(w);
#endif
}

// Burst-wide flags raised inside a grid-stride loop: each lane gathers its
// bits over the loop (flags), the workgroup ORs them in LDS after it, and one
// lane raises each word (flag_once) -- one access per workgroup, where a
// per-wave access per iteration queued tens of thousands of accesses to one
// word.  Every thread of the workgroup calls it once, after its loop.
__device__ __forceinline__ void flags_block(uint32_t *s_fl, uint32_t fl, uint32_t *const *words, int nw) {
#ifdef DP_EMU
  for (int k = 0; k < nw; k++) if (fl & (1u << k)) flag_once(words[k]);
#else
  if (fl) atomicOr(s_fl, fl);
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 0; k < nw; k++)
      if (*s_fl & (1u << k)) flag_once(words[k]);
#endif
}

// Could this record's packet be given a tuple (an expose covers its initial
// source) while its initial destination is a public address of the
// allocator?  Then its initial key may be the reverse key of a pair another
// record creates this burst, and the allocating lane's order would matter
// beyond it: the burst runs on one lane.
__device__ bool masq_back(const dpf::FlowCtx &fc, const dpf::PfReq &R) {
  if (!fc.mq) return false;
  const dpm::View V{fc.mq};
  dpf::FKey ik;
  const uint32_t fam = (R.proto >> 8) & 0xffu;
  const uint32_t kind = (R.bits & dpf::kPqTcp) ? DP_FLOW_TCP : (R.bits & dpf::kPqUdp) ? DP_FLOW_UDP : DP_FLOW_ICMP_QUERY;
  if (R.bits & dpf::kPqIkey) {
    for (int j = 0; j < 11; j++) ik.w[j] = R.ikey[j];
  } else {
    ik.w[1] = fam | (kind << 8);
    for (int j = 0; j < 4; j++) { ik.w[3 + j] = bswap(R.src[j]); ik.w[7 + j] = bswap(R.dst[j]); }
  }
  const uint32_t ifam = ik.w[1] & 0xffu, ikind = ik.w[1] >> 8;
  dpm::A128 d{};
  if (ifam == 4) d.w[3] = bswap(ik.w[7]);
  else for (int j = 0; j < 4; j++) d.w[j] = bswap(ik.w[7 + j]);
  bool pub = false;
  const dpm::Region *G = V.regions();
  for (uint32_t k = 0; k < V.h().n_regions && !pub; k++)
    pub = G[k].fam == ifam && dpm::a_cmp(G[k].start, d) <= 0 && dpm::a_cmp(d, G[k].last) <= 0;
  if (!pub) return false;
  const uint32_t iproto = ikind == DP_FLOW_TCP ? 6u : ikind == DP_FLOW_UDP ? 17u : ifam == 4 ? 1u : 58u;
  dpm::A128 a{};
  if (ifam == 4) a.w[3] = bswap(ik.w[3]);
  else for (int j = 0; j < 4; j++) a.w[j] = bswap(ik.w[3 + j]);
  return dpm::lookup(V, iproto | (ifam << 8), R.src_vni, R.dst_vni, a) != dpm::kNone;
}

// The masquerading record's connection: the lower slot of the flow pair it is
// attached to (the pair's two flows name each other while both live); false:
// no live attached flow (the record goes to the allocating lane).
__device__ bool masq_conn(const dpf::FlowCtx &fc, const dpf::PfReq &R, uint32_t &key) {
  if (R.slot > fc.mask || fc.slots[R.slot].state != R.state) return false;
  const dpf::FlowSlot &A = fc.slots[R.slot];
  key = R.slot;
  if (A.related <= fc.mask && fc.slots[A.related].state == A.related_tag && A.related < key) key = A.related;
  return true;
}

// A record for the allocating lane: its bit by packet index (dp_bits_*, which 1)
__device__ __forceinline__ void lane_mark(const dpf::FlowCtx &fc, dpf::PfReq &R, uint32_t more) {
  R.bits |= dpf::kPqLane | more;
  const uint32_t i = R.idx;
  atomicOr(&fc.lane_bits[i >> 5], 1u << (i & 31));
  uint32_t *sw = &fc.lane_sum[i >> 15];
  const uint32_t sb = 1u << ((i >> 10) & 31);
  if (!(__hip_atomic_load(sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & sb)) atomicOr(sw, sb);
}

// A record's leading words (through dst_vni: what the burst-wide NAT kernels
// read of it; the fields after it are left undefined) and a flow slot, read
// into registers at once.  The empty asm takes every word where the loads are
// issued, so the compiler cannot sink them to their uses: a line read again
// later, with a chip's worth of lanes in flight, has mostly left L2 and is
// fetched from memory again.
__device__ __forceinline__ dpf::PfReq load_req(const dpf::PfReq *p) {
  constexpr int kW = (int)((offsetof(dpf::PfReq, dst_vni) + 4 + 7) / 8);
  uint2 w[kW];
  const uint2 *q = reinterpret_cast<const uint2 *>(p);
#pragma unroll
  for (int i = 0; i < kW; i++) w[i] = q[i];
#ifndef DP_EMU
#pragma unroll
  for (int i = 0; i < kW; i++) asm volatile("" : "+v"(w[i].x), "+v"(w[i].y));
#endif
  dpf::PfReq R;
  __builtin_memcpy(&R, w, sizeof w);
  return R;
}
__device__ __forceinline__ dpf::FlowSlot load_slot(const dpf::FlowSlot *p) {
  uint4 w[8];
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = q[i];
#ifndef DP_EMU
#pragma unroll
  for (int i = 0; i < 8; i++) asm volatile("" : "+v"(w[i].x), "+v"(w[i].y), "+v"(w[i].z), "+v"(w[i].w));
#endif
  dpf::FlowSlot f;
  __builtin_memcpy(&f, w, sizeof w);
  return f;
}

// The words of a flow a steady refresh reads (flags; expiry, pf, pf_rule;
// pf_ip; pf_fam .. nat_tag): four of the slot's eight 16-byte words, the rest
// zero
__device__ __forceinline__ dpf::FlowSlot load_slot_steady(const dpf::FlowSlot *p) {
  static_assert(offsetof(dpf::FlowSlot, flags) / 16 == 3 && offsetof(dpf::FlowSlot, expires_at) / 16 == 5 &&
                offsetof(dpf::FlowSlot, pf_rule) / 16 == 5 && offsetof(dpf::FlowSlot, pf_ip) / 16 == 6 &&
                offsetof(dpf::FlowSlot, pf_fam) / 16 == 7 && offsetof(dpf::FlowSlot, nat_tag) / 16 == 7,
                "the words a steady refresh reads");
  uint4 w[8];
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  w[0] = w[1] = w[2] = w[4] = make_uint4(0u, 0u, 0u, 0u);
  w[3] = q[3]; w[5] = q[5]; w[6] = q[6]; w[7] = q[7];
#ifndef DP_EMU
  for (int i = 3; i < 8; i++)
    if (i != 4) asm volatile("" : "+v"(w[i].x), "+v"(w[i].y), "+v"(w[i].z), "+v"(w[i].w));
#endif
  dpf::FlowSlot f;
  __builtin_memcpy(&f, w, sizeof w);
  return f;
}

// A masquerading record whose refresh leaves its pair's state as it is:
// valid with masquerade state (get_masquerade_state), no ACL flow verdict, a
// NatFlowStatus that the packet does not move (refresh_masquerade_state, nf.rs:
// 151-194, with nw == cur, neither closed nor reset) on a pair that holds a
// live allocation (masq_conn_ok's conditions for the record's own pair).  Its
// outcome is a function of the pair as the burst found it -- if no other
// record of the connection moves the state -- and its one write, the expiry's
// push forward, is a maximum: it commutes with the burst's other records.
// move: the record may move the state (its pair is tagged for the burst).
//
// Over copies of the record, its flow and the flow's related one
// (o: fc.slots[f.related] when f.related <= fc.mask).  The burst-wide kernels
// read each record and flow once into registers: with a chip's worth of lanes
// in flight, a line read again later has mostly left L2 and is fetched again.
__device__ bool masq_steady_v(const dpf::FlowCtx &fc, const dpf::PfReq &R, const dpf::FlowSlot &f,
                              const dpf::FlowSlot &o, bool &move) {
  move = false;
  if ((R.bits & (dpf::kPqMasq | dpf::kPqPf | dpf::kPqSens)) != dpf::kPqMasq) return false;
  if (R.slot > fc.mask || !fc.mq) return false;
  // masq_valid: the attached fill, Active, its pair not invalidated for this
  // packet, with masquerade state
  if (f.state != R.state || R.status0 != DP_FLOW_ACTIVE) return false;
  const bool rel = f.related <= fc.mask && o.state == f.related_tag;
  const uint32_t pi = R.idx + 1;
  if (f.mark <= pi || (rel && o.mark <= pi) || !(f.flags & dpf::kFlagMasq)) return false;
  const uint32_t proto = R.proto & 0xffu, tfl = R.proto >> 16;
  uint32_t src[4], dst[4], sport, dport;
  masq_cur(R, src, dst, sport, dport);
  const uint32_t act = f.pf & 0xffu, cur = (f.pf >> 8) & 0xffu;
  const uint32_t nw = masq_next_status(proto, R.bits & dpf::kPqUdp, sport, tfl, R.bits & dpf::kPqTcp, act, cur);
  if (nw != cur || nw == DP_NFS_CLOSED || nw == DP_NFS_RESET) { move = true; return false; }
  if (!rel) return false;
  if (o.related != R.slot || f.state != o.related_tag || !(o.flags & dpf::kFlagMasq)) return false;
  const dpf::FlowSlot &F = act == DP_PF_SRC_NAT ? f : o, &Rv = act == DP_PF_SRC_NAT ? o : f;
  if ((F.pf & 0xffu) != DP_PF_SRC_NAT || (Rv.pf & 0xffu) != DP_PF_DST_NAT) return false;
  return F.mq_rec && F.mq_gen == fc.mq_gen;
}

// resolve_masq's refresh for a steady record (the expiry by atomicMax); f: a
// copy of its flow
__device__ void masq_steady_run(const dpf::FlowCtx &fc, const dpf::PfReq &Rc, dpf::PfReq &R,
                                const dpf::FlowSlot &f) {
  // (Rc: the record as read -- its bits, slot and proto --, R: where its
  // decision goes -- Masquerade's
  // verdict, action and tuple, 24 contiguous bytes; PortForwarder's verdict
  // and the ACL override keep the values the first pass recorded: a steady
  // record has no port forwarding)
  const uint32_t fam = (Rc.proto >> 8) & 0xffu;
  const bool tcp = Rc.bits & dpf::kPqTcp, udp = Rc.bits & dpf::kPqUdp, icmp = Rc.bits & dpf::kPqIcmp;
  const uint32_t act = f.pf & 0xffu, port = f.pf >> 16, cur = (f.pf >> 8) & 0xffu;
  if (cur != DP_NFS_ONE_WAY) {
    // (every steady record of this flow sees the same status and rule, so
    // writes the same value: a plain store, no atomic)
    const uint64_t ext = cur == DP_NFS_TWO_WAY ? kMasqTwoWayNs
                       : cur == DP_NFS_ESTABLISHED ? (uint64_t)f.pf_rule * 1000000000ull : kMasqClosingNs;
    if (fc.now + ext > f.expires_at) fc.slots[Rc.slot].expires_at = fc.now + ext;
  }
  static_assert(offsetof(dpf::PfReq, mnat) == offsetof(dpf::PfReq, mverdict) + 4 &&
                offsetof(dpf::PfReq, mnat_ip) == offsetof(dpf::PfReq, mverdict) + 8 &&
                offsetof(dpf::PfReq, mverdict) % 8 == 0, "the masquerade decision: 24 contiguous bytes");
  uint2 *d = reinterpret_cast<uint2 *>(&R.mverdict);
  if ((act == DP_PF_SRC_NAT && !unicast(f.pf_fam, f.pf_ip)) || f.pf_fam != fam || !(tcp || udp || icmp)) {
    R.mverdict = DP_DONE_NAT_FAILURE;
    return;
  }
  d[0] = make_uint2(dpf::kPfForward, act | ((f.flags & dpf::kFlagMasqIdent) ? 0x100u : 0u) | (port << 16));
  d[1] = make_uint2(f.pf_ip[0], f.pf_ip[1]);
  d[2] = make_uint2(f.pf_ip[2], f.pf_ip[3]);
}

// A port-forwarding record whose refresh leaves its pair's state as it is
// (round 6): no masquerade, no ACL flow verdict; attached to the fill it found,
// Active, the pair whole (the two flows name each other) and valid for the
// packet, with port-forwarding state whose rule still exists (by_id); a
// NatFlowStatus the packet does not move (refresh_port_fw_entry, flow_state.
// rs:216-264, with nw == cur, neither closed nor reset).  resolve_pf's outcome
// for it is then a function of the pair as the burst found it -- if no other
// record of the connection moves the state, and no creation of the burst
// replaces a flow of the pair (both tag it: dp_nat_mark) -- and its writes (the
// expiry pushed to the same value, the generation) commute with every other
// record's.  Over copies of the record, its flow and the related one.
__device__ bool pf_steady_v(const Img &g, const dpf::FlowCtx &fc, const dpf::PfReq &R, const dpf::FlowSlot &f,
                            const dpf::FlowSlot &o) {
  if ((R.bits & (dpf::kPqMasq | dpf::kPqPf | dpf::kPqSens)) != dpf::kPqPf) return false;
  if (R.slot > fc.mask || f.state != R.state || R.status0 != DP_FLOW_ACTIVE) return false;
  if (f.related > fc.mask || o.state != f.related_tag || o.related != R.slot || o.related_tag != f.state) return false;
  if (f.mark <= R.idx || o.mark <= R.idx || !(f.flags & dpf::kFlagPf)) return false;
  if (by_id(g, f.pf_rule) < 0) return false;
  const uint32_t act = f.pf & 0xffu, cur = (f.pf >> 8) & 0xffu;
  const uint32_t nw = next_status(R.bits & dpf::kPqTcp, R.proto >> 16, act, cur);
  return nw == cur && nw != DP_NFS_CLOSED && nw != DP_NFS_RESET;
}

// resolve_pf for a steady record: the translation from its flow's state, the
// expiry (every steady record of the flow writes the same value: a plain
// store), the flow's generation; f: a copy of its flow
__device__ void pf_steady_run(const Img &g, const dpf::FlowCtx &fc, const dpf::PfReq &Rc, dpf::PfReq &R,
                              const dpf::FlowSlot &f) {
  const int32_t e = by_id(g, f.pf_rule);  // (>= 0: rules do not change within a burst)
  const uint32_t act = f.pf & 0xffu, cur = (f.pf >> 8) & 0xffu;
  R.verdict = dpf::kPfForward;
  R.acl_over = 0;
  R.nat = act | (f.pf & 0xffff0000u);
  for (int j = 0; j < 4; j++) R.nat_ip[j] = f.pf_ip[j];
  const PfRuleRec &E = g.at<PfRuleRec>(g.im.pf_rules)[e];
  const uint64_t nw = fc.now + (cur == DP_NFS_ESTABLISHED ? E.estab_ns : E.init_ns);
  if (nw >= f.expires_at) fc.slots[Rc.slot].expires_at = nw;
  if (f.genid != fc.genid) fc.slots[Rc.slot].genid = fc.genid;
}

// dp_nat_prep's half: the record's flow untagged (no record of the burst
// moves or replaces its pair), then its refresh
__device__ bool pf_steady_here(const Img &g, const dpf::FlowCtx &fc, const dpf::PfReq &Rc, dpf::PfReq &R) {
  const dpf::FlowSlot f = load_slot(&fc.slots[Rc.slot]);
  if (f.nat_tag == fc.burst) return false;
  pf_steady_run(g, fc, Rc, R, f);
  R.bits = Rc.bits | dpf::kPqSteady;
  return true;
}

// Can a connection lane run this connection (the records of `list`)?  Every
// record masquerades without port forwarding, is attached to one of the
// pair's two flows (still the fills it attached) and was Active as the burst
// started; the pair holds masquerade state (the forward flow SrcNat, the
// reverse DstNat) and the forward flow owns a live allocation.
__device__ bool masq_conn_ok(const Seq &q, uint32_t list) {
  const dpf::FlowCtx &fc = q.fc;
  if (!fc.mq) return false;
  const uint32_t S = fc.pf[list].slot;
  if (S > fc.mask) return false;
  const dpf::FlowSlot &A = fc.slots[S];
  if (!q.alive(A.related, A.related_tag)) return false;
  const uint32_t T = A.related;
  const dpf::FlowSlot &B = fc.slots[T];
  if (B.related != S || !q.alive(S, B.related_tag)) return false;
  if (!(A.flags & dpf::kFlagMasq) || !(B.flags & dpf::kFlagMasq)) return false;
  const bool a_fw = (A.pf & 0xffu) == DP_PF_SRC_NAT;
  const dpf::FlowSlot &F = a_fw ? A : B, &Rv = a_fw ? B : A;
  if ((F.pf & 0xffu) != DP_PF_SRC_NAT || (Rv.pf & 0xffu) != DP_PF_DST_NAT) return false;
  if (!F.mq_rec || F.mq_gen != fc.mq_gen) return false;
  for (uint32_t r = list; r != dpf::kNoSlot; r = (uint32_t)link_ld(&fc.grp_next[r])) {
    const dpf::PfReq &R = fc.pf[r];
    if ((R.bits & (dpf::kPqMasq | dpf::kPqPf)) != dpf::kPqMasq) return false;
    if ((R.slot != S && R.slot != T) || !q.alive(R.slot, R.state) || R.status0 != DP_FLOW_ACTIVE) return false;
  }
  return true;
}

// One masquerading connection on its lane (dp_nat_resolve, mode 3).
__device__ void masq_conn_run(const Seq &q, uint32_t list) {
  const dpf::FlowCtx &fc = q.fc;
  bool lane = !masq_conn_ok(q, list);
  for (uint32_t r = list; r != dpf::kNoSlot; r = (uint32_t)link_ld(&fc.grp_next[r])) {
    dpf::PfReq &R = fc.pf[r];
    if (lane) { lane_mark(fc, R, 0u); continue; }
    R.mverdict = dpf::kPfForward;
    resolve_pf(q, R);  // (no port forwarding here: the ACL's flow verdict only)
    if (R.verdict != dpf::kPfForward) continue;
    if (masq_valid(q, R)) { resolve_masq(q, R); continue; }
    // the flow is no longer valid for it: it allocates, on the allocating lane
    lane_mark(fc, R, dpf::kPqPfDone);
    atomicAdd(&fc.pf_cnt[13], 1u);
    lane = true;
  }
}

// ---------------------------------------------------------------------------
// Port forwarding near the capacity (mode 4)
// ---------------------------------------------------------------------------
// insert_common refuses a flow when the table holds `capacity` flows (the
// second of a pair excepted), so once the burst's creations fill the table,
// every later creation in packet order is refused; before that point every
// one is admitted.  Which one first meets the capacity follows from how many
// new slots each creation adds, summed in packet order -- known before any
// runs when each connection's creations are: a connection whose records are
// all without a flow (its first creation adds a slot for each of its two
// keys not in the table, a repeat replaces those), or one that creates
// nothing (each record that could is on a valid flow with port-forwarding
// state whose rule lives, and no earlier record of it can close the pair).
// Any other connection (pf_cnt[17]) leaves the burst to the one-lane pass.

// A record on its connection's valid port-forwarding pair, which refreshes
// rather than creates (resolve_pf's first branch, no rule to revalidate, no
// ACL flow verdict)
__device__ bool pf_held(const Seq &q, const dpf::PfReq &R) {
  if (R.slot == dpf::kNoSlot || !q.alive(R.slot, R.state) || R.status0 != DP_FLOW_ACTIVE) return false;
  if ((R.bits & dpf::kPqSens) || !q.pair_valid(R.slot, R.idx)) return false;
  const dpf::FlowSlot &f = q.fc.slots[R.slot];
  return (f.flags & dpf::kFlagPf) && by_id(q.g, f.pf_rule) >= 0;
}

// The creation's forward key (resolve_pf: the key before static NAT, else the
// current one)
__device__ void creation_fk(const dpf::PfReq &R, dpf::FKey &fk) {
  if (R.bits & dpf::kPqIkey) {
    for (int j = 0; j < 11; j++) fk.w[j] = R.ikey[j];
  } else {
    const uint32_t fam = (R.proto >> 8) & 0xffu;
    fk.w[0] = R.src_vni;
    fk.w[1] = fam | (((R.bits & dpf::kPqTcp) ? DP_FLOW_TCP : DP_FLOW_UDP) << 8);
    fk.w[2] = R.ports;
    for (int j = 0; j < 4; j++) { fk.w[3 + j] = bswap(R.src[j]); fk.w[7 + j] = bswap(R.dst[j]); }
  }
}

// One connection (its records sorted): fc.adm[record] = the new slots its
// creation adds; false: its creations cannot be foreseen.
__device__ bool admit_plan(const Seq &q, uint32_t list) {
  const dpf::FlowCtx &fc = q.fc;
  bool pure = true, held = true, closing = false;
  for (uint32_t r = list; r != dpf::kNoSlot; r = (uint32_t)link_ld(&fc.grp_next[r])) {
    const dpf::PfReq &R = fc.pf[r];
    dpf::FKey rk;
    const bool cand = creation_rk(q.g, R, rk), h = pf_held(q, R);
    if (R.slot != dpf::kNoSlot) pure = false;
    if (cand && (closing || !h)) held = false;
    // a record after which the pair may be invalid: a TCP FIN / RST, the ACL's
    // flow verdict, a flow that is not held (a rule to revalidate, ...)
    if (((R.bits & dpf::kPqTcp) && ((R.proto >> 16) & 5u)) || (R.bits & dpf::kPqSens) ||
        (R.slot != dpf::kNoSlot && !h))
      closing = true;
  }
  if (!pure && !held) return false;
  // (a group may hold several connections -- keys that collide in the hash
  // merge them: a creation adds slots unless an earlier one of the group
  // made the same pair)
  for (uint32_t r = list; r != dpf::kNoSlot; r = (uint32_t)link_ld(&fc.grp_next[r])) {
    const dpf::PfReq &R = fc.pf[r];
    uint32_t w = 0;
    dpf::FKey rk, fk;
    if (pure && creation_rk(q.g, R, rk)) {
      bool again = false;
      for (uint32_t p = list; p != r && !again; p = (uint32_t)link_ld(&fc.grp_next[p])) {
        dpf::FKey pk;
        if (!creation_rk(q.g, fc.pf[p], pk)) continue;
        again = true;
        for (int j = 0; j < 11; j++) again = again && pk.w[j] == rk.w[j];
      }
      if (!again) {
        creation_fk(R, fk);
        uint32_t st;
        uint4 v, x;
        w = (flow_probe(fc, fk, st, v, x) == dpf::kNoSlot ? 1u : 0u) +
            (flow_probe(fc, rk, st, v, x) == dpf::kNoSlot ? 1u : 0u);
      }
    }
    fc.adm[r] = w;
  }
  return true;
}

}  // namespace pfw

#if DP_IN_PART(0)
// The packets a bitmap marks (by packet index, 1024 per summary bit) in
// packet order, in three launches: each 1024-packet region's count (one
// work-item per region, its 32 words), their exclusive prefix (one
// workgroup), each region's packets written at its offset (one wave per
// region, a lane per word); the bits are cleared for the next burst.
// which: 0 the NAT stages' packets (pf_bits -> pf_order, pf_cnt[1], and the
// table length as the pass starts in pf_cnt[6..7]), 1 the allocating lane's
// (lane_bits -> lane_order, pf_cnt[11]).  The region counts live in adm (per
// 1024 packets, free until dp_nat_admit_plan).
__global__ void __launch_bounds__(256) dp_bits_count(dpf::FlowCtx fc, int which) {
  const uint32_t *bits = which ? fc.lane_bits : fc.pf_bits, *sum = which ? fc.lane_sum : fc.pf_sum;
  const uint32_t regions = (fc.n + 1023) / 1024;
  for (uint32_t r = blockIdx.x * 256 + threadIdx.x; r < regions; r += gridDim.x * 256) {
    uint32_t c = 0;
    if ((sum[r >> 5] >> (r & 31)) & 1u) {
      const uint4 *w = reinterpret_cast<const uint4 *>(bits + 32 * (uint64_t)r);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint4 x = w[j];
        c += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
      }
    }
    fc.adm[r] = c;
  }
}
__global__ void __launch_bounds__(1024) dp_bits_scan(dpf::FlowCtx fc, int which) {
  const uint32_t t = threadIdx.x, regions = (fc.n + 1023) / 1024;
  __shared__ uint32_t sh[1024];
  __shared__ uint32_t base;
  if (t == 0) base = 0;
  for (uint32_t r0 = 0; r0 < regions; r0 += 1024) {
    __syncthreads();
    const uint32_t v = r0 + t < regions ? fc.adm[r0 + t] : 0u;
    sh[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
      const uint32_t x = t >= o ? sh[t - o] : 0u;
      __syncthreads();
      sh[t] += x;
      __syncthreads();
    }
    if (r0 + t < regions) fc.adm[r0 + t] = base + sh[t] - v;
    __syncthreads();
    if (t == 1023) base += sh[1023];
  }
  __syncthreads();
  if (t == 0) {
    if (which) {
      fc.pf_cnt[11] = base;
    } else {
      fc.pf_cnt[1] = base;
      fc.pf_cnt[6] = fc.tmeta[2];  // the table length before the pass
      fc.pf_cnt[7] = fc.tmeta[3];
    }
  }
}
__global__ void __launch_bounds__(256) dp_bits_emit(dpf::FlowCtx fc, int which) {
  uint32_t *bits = which ? fc.lane_bits : fc.pf_bits, *sum = which ? fc.lane_sum : fc.pf_sum;
  uint32_t *order = which ? fc.lane_order : fc.pf_order;
  const uint32_t regions = (fc.n + 1023) / 1024, lane = threadIdx.x & 63;
  for (uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6); r < regions; r += gridDim.x * 4) {
    if (!((sum[r >> 5] >> (r & 31)) & 1u)) continue;  // (uniform per wave)
    const uint32_t w = lane < 32 ? bits[32 * (uint64_t)r + lane] : 0u;
    // the word's offset in the region: the words before it (wave prefix)
    uint32_t c = (uint32_t)__popc(w), x = c;
    for (int o = 1; o < 32; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if ((int)lane >= o) x += y;
    }
    uint32_t pos = fc.adm[r] + x - c;
    if (w) {
      bits[32 * (uint64_t)r + lane] = 0;
      for (uint32_t b = w; b; b &= b - 1) order[pos++] = r * 1024 + lane * 32 + (uint32_t)(__ffs(b) - 1);
    }
  }
}
// (then the summary words, once every region is emitted)
__global__ void __launch_bounds__(256) dp_bits_clear(dpf::FlowCtx fc, int which) {
  uint32_t *sum = which ? fc.lane_sum : fc.pf_sum;
  const uint32_t words = ((fc.n + 1023) / 1024 + 31) / 32;
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < words; k += gridDim.x * 256) sum[k] = 0;
}

// dp_nat_mark: the burst's kinds of record (port forwarding, masquerade, a
// peer that could masquerade back: the NAT pass's mode), and every
// masquerading record that is not a steady refresh (pfw::masq_steady) tags
// its flow pair for the burst: that connection's records run in its order
// (dp_nat_prep files them), not as steady ones.
__global__ void __launch_bounds__(256) dp_nat_mark(const uint8_t *__restrict__ img_base,
                                                   const Image *__restrict__ im, dpf::FlowCtx fc) {
  const uint32_t nrec = fc.pf_cnt[0];
  if (!nrec) return;
  const Img g{img_base, *im};
  __shared__ uint32_t s_fl;
  if (threadIdx.x == 0) s_fl = 0;
  __syncthreads();
  // the kinds seen: 1 port forwarding, 2 masquerade, 4 masq_back, 8 what a
  // mixed burst cannot run beside the split (a record that both forwards and
  // masquerades, a masquerading record on a port-forwarded flow)
  uint32_t fl = 0;
  for (uint32_t rec = blockIdx.x * 256 + threadIdx.x; rec < nrec; rec += gridDim.x * 256) {
    // the record's kinds; a steady refresh (its bit in fc.steady, a word per
    // wave: the wave's 64 records are consecutive), else its pair's tag
    auto visit = [&]() -> bool {
      const dpf::PfReq R = pfw::load_req(&fc.pf[rec]);  // (the record, its flow and the related flow read once)
      // the burst's kinds of record (the NAT pass's mode rests on them)
      if (!(R.bits & dpf::kPqReached)) return false;
      if (R.bits & dpf::kPqPf) fl |= 1u;
      if (!(R.bits & dpf::kPqMasq)) {
        // a port-forwarding steady refresh (pfw::pf_steady_v); any other
        // record tags the pair it is attached to -- a port-forwarding record
        // on a masqueraded pair (a creation replaces its flow) too: that
        // pair's refreshes are not order-free -- and a creation the pair whose
        // reverse flow holds its reverse key (it replaces that flow).  Such a
        // pair has another forward key than the creation's (the creation's
        // own would have been found and attached), which only rules whose
        // internal sides overlap allow (Image.pf_overlap); a pair whose
        // forward flow is gone is never steady (pf_steady_v wants it whole)
        if (R.slot <= fc.mask) {
          const dpf::FlowSlot f = pfw::load_slot(&fc.slots[R.slot]);
          if (f.state == R.state) {
            dpf::FlowSlot o;
            if (f.related <= fc.mask) o = pfw::load_slot(&fc.slots[f.related]);
            else o.state = 0;
            if (pfw::pf_steady_v(g, fc, R, f, o)) return true;
            fc.slots[R.slot].nat_tag = fc.burst;
            if (f.related <= fc.mask && o.state == f.related_tag) fc.slots[f.related].nat_tag = fc.burst;
          }
        }
        dpf::FKey rk;
        if ((R.bits & dpf::kPqPf) && g.im.pf_overlap && pfw::creation_rk(g, R, rk)) {
          uint32_t st;
          uint4 v, w;
          const uint32_t z = flow_probe(fc, rk, st, v, w);
          if (z != dpf::kNoSlot) {
            fc.slots[z].nat_tag = fc.burst;
            const uint32_t zr = fc.slots[z].related;
            if (zr <= fc.mask && fc.slots[zr].state == fc.slots[z].related_tag) fc.slots[zr].nat_tag = fc.burst;
          }
        }
        return false;
      }
      fl |= 2u;
      if (R.bits & dpf::kPqPf) fl |= 8u;
      if (!(fl & 4u) && pfw::masq_back(fc, R)) fl |= 4u;
      if (!fc.mq || R.slot > fc.mask) return false;
      const dpf::FlowSlot f = pfw::load_slot(&fc.slots[R.slot]);
      if (f.state != R.state) return false;
      if (f.flags & dpf::kFlagPf) fl |= 8u;
      dpf::FlowSlot o;
      if (f.related <= fc.mask) o = pfw::load_slot(&fc.slots[f.related]);
      else o.state = 0;
      bool move;
      if (pfw::masq_steady_v(fc, R, f, o, move)) return true;
      fc.slots[R.slot].nat_tag = fc.burst;
      if (f.related <= fc.mask && o.state == f.related_tag) fc.slots[f.related].nat_tag = fc.burst;
      return false;
    };
    const bool st = visit();
#ifdef DP_EMU
    if (st) fc.steady[rec >> 6] |= 1ull << (rec & 63);
    else fc.steady[rec >> 6] &= ~(1ull << (rec & 63));
#else
    const uint64_t m = __ballot(st);
    if ((threadIdx.x & 63) == 0) fc.steady[rec >> 6] = m;
#endif
  }
  uint32_t *const words[4] = {&fc.pf_cnt[9], &fc.pf_cnt[8], &fc.pf_cnt[10], &fc.pf_cnt[30]};
  pfw::flags_block(&s_fl, fl, words, 4);
}

// dp_nat_prep: the records of the burst's NAT pass (their packet order for
// the one-lane pass and the replay: dp_bits_*); each record is filed under its
// connection -- port forwarding: pfw::conn_key; masquerade: the flow pair it is
// attached to (pfw::masq_conn), or the allocating lane -- a hash slot claimed
// for this burst by CAS on (burst, key), a list of its records pushed by CAS
// on (burst, last record).
__global__ void __launch_bounds__(1024) dp_nat_prep(const uint8_t *__restrict__ img_base,
                                                    const Image *__restrict__ im, dpf::FlowCtx fc) {
  const uint32_t t = threadIdx.x;
  const uint32_t nrec = fc.pf_cnt[0];
  if (!nrec) return;
  const Img g{img_base, *im};
  const uint32_t mode0 = pfw::nat_mode(fc);  // (dp_nat_mark's flags decide it)
  const bool split = pfw::split_mode(mode0), mixed = mode0 == 5;
  // (port-forwarding steady refreshes: the connection lanes' modes without
  // admissions -- mode 4 counts its creations' slots over whole connections)
  const bool pfsteady = mode0 == 2 || mode0 == 5;
  const unsigned long long tag = (unsigned long long)fc.burst << 32;
  __shared__ uint32_t s_fl;
  if (t == 0) s_fl = 0;
  __syncthreads();
  uint32_t fl = 0;  // 1 a steady refresh, 2 a record the parallel pass cannot place
  // the connections new this burst: their list entries claimed once per
  // workgroup and pass (a claim per wave queued ~10k same-word atomics)
  __shared__ uint32_t s_cnt[16], s_base;
  // a mixed burst: a bound on the slots its inserts may add (pf_cnt[31]) --
  // two per port-forwarding connection (its creations insert the same two
  // keys) and two per masquerading record that is not a steady refresh (an
  // allocation inserts its initial key and a new reverse key)
  __shared__ uint32_t s_add;
  if (t == 0) s_add = 0;
  uint32_t add = 0;
  // file one record; fresh: its connection is new (h: its hash slot)
  auto visit = [&](uint32_t rec, uint32_t &h, bool &fresh) {
    dpf::PfReq &R = fc.pf[rec];
    // (the record's first words: bits, slot, state ... proto, read at once)
    dpf::PfReq Rc;
    {
      const uint2 *q = reinterpret_cast<const uint2 *>(&R);  // (records are 8-byte aligned)
      uint2 w[4] = {q[0], q[1], q[2], q[3]};
#ifndef DP_EMU
      for (int i = 0; i < 4; i++) asm volatile("" : "+v"(w[i].x), "+v"(w[i].y));
#endif
      static_assert(offsetof(dpf::PfReq, proto) < 32, "bits, slot and proto in the first 32 bytes");
      __builtin_memcpy(&Rc, w, sizeof w);
    }
    if (!(Rc.bits & dpf::kPqReached)) return;  // a flow-filter record of a packet dropped before NAT
    uint32_t key;
    if (Rc.bits & dpf::kPqMasq) {
      // a steady refresh (dp_nat_mark) whose connection no record moves (its
      // flow untagged: a tag reaches both flows of the pair): resolved here
      // (split pass; the one-lane pass runs it in its order) from its flow
      // alone
      if (split && ((fc.steady[rec >> 6] >> (rec & 63)) & 1u)) {
        const dpf::FlowSlot f = pfw::load_slot_steady(&fc.slots[Rc.slot]);
        if (f.nat_tag != fc.burst) {
          fl |= 1u;
          pfw::masq_steady_run(fc, Rc, R, f);
          R.bits = Rc.bits | dpf::kPqSteady;
          return;
        }
      }
      if (mixed) add += 2;
      if (!pfw::masq_conn(fc, R, key)) {
        pfw::lane_mark(fc, R, 0u);
        return;
      }
    } else if (pfsteady && ((fc.steady[rec >> 6] >> (rec & 63)) & 1u) &&
               pfw::pf_steady_here(g, fc, Rc, R)) {
      // a port-forwarding steady refresh whose pair no record moves: resolved
      // here (the one-lane pass, should the burst fall back to it, runs it
      // again in its order, to the same outcome)
      fl |= 1u;
      return;
    } else if (pfw::conn_key(g, fc, R, key, mixed)) {
      key |= pfw::kPfConnBit;
    } else {
      fl |= 2u;
      return;
    }
    const unsigned long long want = tag | key;
    h = dpm::kmix(key, 0x2545f491u, 0u) & fc.grp_mask;
    for (uint32_t p = 0; p <= fc.grp_mask;) {
      const unsigned long long cur = __hip_atomic_load(&fc.grp_tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == want) break;
      if ((cur >> 32) == fc.burst) { h = (h + 1) & fc.grp_mask; p++; continue; }
      if (atomicCAS(&fc.grp_tab[h], cur, want) == cur) {
        fresh = true;
        break;
      }
    }
    unsigned long long old = __hip_atomic_load(&fc.grp_head[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      const uint32_t prev = (old >> 32) == fc.burst ? (uint32_t)old : dpf::kNoSlot;
      fc.grp_next[rec] = ((unsigned long long)R.idx << 32) | prev;
      const unsigned long long got = atomicCAS(&fc.grp_head[h], old, tag | rec);
      if (got == old) break;
      old = got;
    }
  };
  for (uint32_t b0 = blockIdx.x * 1024; b0 < nrec; b0 += gridDim.x * 1024) {  // (uniform per workgroup)
    const uint32_t rec = b0 + t;
    uint32_t h = 0;
    bool fresh = false;
    if (rec < nrec) visit(rec, h, fresh);
    if (mixed && fresh && (fc.grp_tab[h] & pfw::kPfConnBit)) add += 2;
#ifdef DP_EMU
    if (fresh) fc.grp_list[atomicAdd(&fc.pf_cnt[4], 1u)] = h;
#else
    const uint64_t m = __ballot(fresh);
    const uint32_t wv = t >> 6;
    if ((t & 63) == 0) s_cnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (t == 0) {
      uint32_t sum = 0;
      for (int k = 0; k < 16; k++) { const uint32_t c = s_cnt[k]; s_cnt[k] = sum; sum += c; }
      s_base = sum ? atomicAdd(&fc.pf_cnt[4], sum) : 0u;
    }
    __syncthreads();
    if (fresh) fc.grp_list[s_base + s_cnt[wv] + (uint32_t)__popcll(m & lanes_below((int)(t & 63)))] = h;
    __syncthreads();
#endif
  }
  if (mixed) {
#ifdef DP_EMU
    if (add) atomicAdd(&fc.pf_cnt[31], add);
#else
    if (add) atomicAdd(&s_add, add);
    __syncthreads();
    if (t == 0 && s_add) atomicAdd(&fc.pf_cnt[31], s_add);
#endif
  }
  uint32_t *const words[2] = {&fc.pf_cnt[27], &fc.pf_cnt[5]};
  pfw::flags_block(&s_fl, fl, words, 2);
}

// dp_nat_cross (mode 5): a masquerading record without a live attached flow
// may allocate, and its pair's first insert is its initial key; when that is
// the reverse key of a port-forwarding creation of the burst (dp_nat_prep
// registered them), the allocating lane and the connection lanes would meet
// in one key: the burst runs on one lane (pf_cnt[30]).  A record on a live
// flow needs no look: its initial key is that flow's, which a creation's
// reverse key cannot be (conn_key).
__global__ void __launch_bounds__(256) dp_nat_cross(dpf::FlowCtx fc) {
  const uint32_t nrec = fc.pf_cnt[0];
  if (!nrec || !fc.pf_cnt[1] || pfw::nat_mode(fc) != 5) return;
  __shared__ uint32_t s_fl;
  if (threadIdx.x == 0) s_fl = 0;
  __syncthreads();
  uint32_t fl = 0, looked = 0, found = 0;
  // (the record read in place: a copy through load_req gave wrong keys in
  // this kernel's optimised build -- an unexplained codegen interaction;
  // DESIGN.md §3)
  for (uint32_t rec = blockIdx.x * 256 + threadIdx.x; rec < nrec; rec += gridDim.x * 256) {
    const dpf::PfReq &R = fc.pf[rec];
    // (a steady refresh dp_nat_prep resolved has its live flow: no slot read)
    if ((R.bits & (dpf::kPqReached | dpf::kPqMasq | dpf::kPqSteady)) != (dpf::kPqReached | dpf::kPqMasq)) continue;
    if (R.slot <= fc.mask && fc.slots[R.slot].state == R.state) continue;
    dpf::FKey ik;
    if (!pfw::masq_ik(R, ik)) continue;
    looked++;
    if (pfw::cross_has(fc, ik)) { fl = 1u; found++; }
  }
  if (looked) atomicAdd(&fc.pf_cnt[33], looked);
  if (found) atomicAdd(&fc.pf_cnt[34], found);
  uint32_t *const words[1] = {&fc.pf_cnt[30]};
  pfw::flags_block(&s_fl, fl, words, 1);
}

// dp_nat_resolve: the reference's PortForwarder and Masquerade over the
// records -- NatFlowStatus, expiries, invalidation marks and events, rule
// revalidation, allocations, the inserts of new pairs -- leaving each
// packet's decision in its record for the replay pass.  Mode 2 (port
// forwarding): one lane per connection (its records in packet order), when no
// record needs the one-lane pass and no insert of the burst can meet the
// capacity or the 7/8 bound (the admissions of insert_common,
// flow-entry/src/flow_table/table.rs:215-260, then cannot depend on the
// order of connections).  Mode 3 (masquerade): the connection lanes of the
// split pass (above).  Mode 1: one lane over all records in packet order.
// Two instantiations, one launch each: SEQ (one wave) runs mode 1, the other
// (the grid) modes 2 and 3; each leaves at once otherwise.  Apart, each is
// compiled for its own mode: the sequential lane's records inlined (no call
// frame to save and restore per record), the parallel lanes at 6 waves per
// SIMD.
#ifndef DP_RESOLVE_WAVES
#define DP_RESOLVE_WAVES 6
#endif
template <bool SEQ>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEQ ? 1 : DP_RESOLVE_WAVES)))
dp_nat_resolve(const uint8_t *__restrict__ img_base, const Image *__restrict__ im, dpf::FlowCtx fc) {
  const uint32_t total = fc.pf_cnt[1];
  if (!total) return;
  const Img g{img_base, *im};
  const uint32_t mode = pfw::nat_mode(fc);
  if ((mode == 1) != SEQ) return;
  const uint32_t gt = blockIdx.x * 256 + threadIdx.x;
  if (gt == 0) fc.pf_cnt[12] = mode;
  if constexpr (SEQ) {
    // one lane in packet order; the other 63 lanes of its wave run ahead,
    // loading what the next 64 records will read -- the record, its flow and
    // that flow's related flow, the home slot of the key a creation inserts
    // first -- so the lane's chain of dependent accesses meets L2 lines
    // instead of HBM ones (values unused: the loads only warm the cache)
    if (gt >= 64) return;
    const pfw::Seq q{fc, g, false};
    for (uint32_t k0 = 0; k0 < total; k0 += 64) {
      if (k0 + gt < total) {
        const dpf::PfReq &P = fc.pf[fc.pf_of[fc.pf_order[k0 + gt]]];
        uint32_t acc = P.bits ^ P.proto;
        if (P.slot <= fc.mask) {
          const uint4 a = ld4(&fc.slots[P.slot].state);
          acc ^= a.x;
          if (P.related0 <= fc.mask) acc ^= ld4(&fc.slots[P.related0].state).x;
        }
        dpf::FKey k;
        if (P.bits & dpf::kPqIkey) {
          for (int j = 0; j < 11; j++) k.w[j] = P.ikey[j];
        } else {
          const uint32_t kind = (P.bits & dpf::kPqTcp) ? DP_FLOW_TCP : (P.bits & dpf::kPqUdp) ? DP_FLOW_UDP
                                                                                         : DP_FLOW_ICMP_QUERY;
          k.w[0] = P.src_vni;
          k.w[1] = ((P.proto >> 8) & 0xffu) | (kind << 8);
          k.w[2] = P.ports;
          for (int j = 0; j < 4; j++) { k.w[3 + j] = pfw::bswap(P.src[j]); k.w[7 + j] = pfw::bswap(P.dst[j]); }
        }
        acc ^= ld4(&fc.slots[dpf::fkey_hash(k) & fc.mask].state).x;
        asm volatile("" ::"v"(acc));
      }
      if (gt == 0)
        for (uint32_t k = k0; k < total && k < k0 + 64; k++) pfw::resolve_one(q, fc.pf[fc.pf_of[fc.pf_order[k]]]);
    }
    // the flows replaced during the burst are dropped after it, with the
    // allocations their masquerade state owns (by the one lane)
    if (gt == 0 && fc.mq) {
      const dpm::View V{fc.mq};
      for (uint32_t k = 0; k < fc.pf_cnt[3]; k++) dpm::release(V, fc.mq_rel[2 * k], fc.mq_rel[2 * k + 1]);
    }
    return;
  }
  const pfw::Seq q{fc, g, true};
  const uint32_t ng = fc.pf_cnt[4];
  for (uint32_t e = gt; e < ng; e += gridDim.x * 256) {
    const uint32_t h = fc.grp_list[e];
#ifdef DP_DEBUG_NAT_NOSORT
    uint32_t r = (uint32_t)fc.grp_head[h];
#else
    // (mode 4: dp_nat_admit_plan sorted the list already)
    uint32_t r = mode == 4 ? (uint32_t)fc.grp_head[h] : pfw::sort_conn(fc.grp_next, (uint32_t)fc.grp_head[h]);
#endif
    // (mode 5: a masquerading connection, or a port-forwarding one -- never
    // both: their keys differ in bit 31)
    if (mode == 3 || (mode == 5 && (fc.pf[r].bits & dpf::kPqMasq))) {
      pfw::masq_conn_run(q, r);
      continue;
    }
    for (; r != dpf::kNoSlot; r = (uint32_t)pfw::link_ld(&fc.grp_next[r])) {
#ifdef DP_DEBUG_NAT
      fc.pf[r].mnat_ip[0] = e;
      atomicAdd(&fc.pf[r].mnat_ip[1], 1u);
#endif
      if (mode == 4) q.adm = fc.adm[r];
      pfw::resolve_one(q, fc.pf[r]);
    }
  }
  // the table length, one add per wave (every lane of the wave is here)
  uint32_t v = q.added;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0 && v)
    atomicAdd(reinterpret_cast<unsigned long long *>(&fc.tmeta[2]), (unsigned long long)v);
}

// dp_nat_admit_plan (mode 4): each connection's creations and the new slots
// each adds (pfw::admit_plan), or pf_cnt[17]: the burst runs on one lane.
__global__ void __launch_bounds__(256) dp_nat_admit_plan(const uint8_t *__restrict__ img_base,
                                                         const Image *__restrict__ im, dpf::FlowCtx fc) {
  if (!fc.pf_cnt[1] || pfw::nat_mode(fc, true) != 4) return;
  const Img g{img_base, *im};
  const pfw::Seq q{fc, g, true};
  const uint32_t ng = fc.pf_cnt[4];
  for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < ng; e += gridDim.x * 256) {
    const uint32_t h = fc.grp_list[e];
    const uint32_t r = pfw::sort_conn(fc.grp_next, (uint32_t)fc.grp_head[h]);
    // (the sorted list's head, for dp_nat_resolve)
    fc.grp_head[h] = ((unsigned long long)fc.burst << 32) | r;
    if (!pfw::admit_plan(q, r)) pfw::flag_once(&fc.pf_cnt[17]);
  }
}

// dp_nat_admit_scan (mode 4): the new slots of the records before each, in
// packet order -- three launches: (0) each 4096 records' sum, (1) their
// exclusive prefix, (2) each record's.
constexpr uint32_t kAdmChunk = 4096;
__global__ void __launch_bounds__(1024) dp_nat_admit_scan(dpf::FlowCtx fc, int step) {
  if (!fc.pf_cnt[1] || pfw::nat_mode(fc) != 4) return;
  const uint32_t total = fc.pf_cnt[1], t = threadIdx.x;
  __shared__ uint32_t sh[1024];
  if (step == 1) {
    const uint32_t nb = (total + kAdmChunk - 1) / kAdmChunk;  // <= 1024 (n <= 4M)
    const uint32_t v = t < nb ? fc.adm_blk[t] : 0u;
    sh[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
      const uint32_t x = t >= o ? sh[t - o] : 0u;
      __syncthreads();
      sh[t] += x;
      __syncthreads();
    }
    if (t < nb) fc.adm_blk[t] = sh[t] - v;
    return;
  }
  // (the grid covers the burst; only the blocks over records take part, so
  // adm_blk's 1024 words hold any burst size: nat_mode keeps total <= 4M)
  if (blockIdx.x * kAdmChunk >= total) return;
  const uint32_t k0 = blockIdx.x * kAdmChunk + t * 4;
  uint32_t w[4], c = 0;
  for (int j = 0; j < 4; j++) {
    w[j] = k0 + j < total ? fc.adm[fc.pf_of[fc.pf_order[k0 + j]]] : 0u;
    c += w[j];
  }
  sh[t] = c;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint32_t x = t >= o ? sh[t - o] : 0u;
    __syncthreads();
    sh[t] += x;
    __syncthreads();
  }
  if (step == 0) {
    if (t == 1023) fc.adm_blk[blockIdx.x] = sh[1023];
    return;
  }
  uint32_t s = fc.adm_blk[blockIdx.x] + sh[t] - c;
  for (int j = 0; j < 4; j++) {
    if (k0 + j < total) fc.adm[fc.pf_of[fc.pf_order[k0 + j]]] = s;
    s += w[j];
  }
}

// dp_nat_lane_plan: the allocating lane's records planned in parallel before
// it runs: a record whose flow is valid with masquerade state (or carries the
// ACL's flow verdict) runs alone, on live state; so do all when the table
// lacks room for every pair the lane could create; the others are decided
// without the allocator or ask it for a tuple (masq_plan: configuration only).
// Validity only ever falls during the pass, so a plan made now errs only
// towards "alone", which re-decides live.  Each wave plans one 64-record
// chunk of the lane (the lane's unit) and finds, per allocating record, the
// latest earlier one of the chunk with the same initial key (its pair replaces
// that one's: the lane cuts its runs there); burst-wide, pf_cnt[28] says
// some initial key repeats, pf_cnt[29] that some record runs alone -- without
// either, every pair commutes with the others and dp_nat_pairs creates them
// after the lane's allocations.
__global__ void __launch_bounds__(256) dp_nat_lane_plan(const uint8_t *__restrict__ img_base,
                                                        const Image *__restrict__ im, dpf::FlowCtx fc) {
  if (!fc.pf_cnt[1] || !pfw::split_mode(pfw::nat_mode(fc))) return;
  const uint32_t nl = fc.pf_cnt[11];
  const Img g{img_base, *im};
  const pfw::Seq qs{fc, g, false};
  const dpm::View V{fc.mq};
  const uint64_t len0 = ((uint64_t)fc.tmeta[3] << 32) | fc.tmeta[2];
  const bool room = len0 + 2ull * nl <= fc.capacity && len0 + 2ull * nl <= fc.hard;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ uint32_t s_ik[4][64][12];
  __shared__ uint32_t s_hc[4][256];
  const unsigned long long tag = (unsigned long long)fc.burst << 32;
  for (uint32_t b0 = blockIdx.x * 256; b0 < nl; b0 += gridDim.x * 256) {  // (uniform per block)
    const uint32_t k = b0 + 64 * wv + lane;
    const bool has = k < nl;
    pfw::LanePlan L{};
    if (has) {
      L.rec = fc.pf_of[fc.lane_order[k]];
      dpf::PfReq &R = fc.pf[L.rec];
      const bool pfdone = R.bits & dpf::kPqPfDone;
      if (!room || (!pfdone && (R.bits & dpf::kPqSens)) || pfw::masq_valid(qs, R)) {
        L.cls = 1;
      } else {
        R.mverdict = dpf::kPfForward;
        if (!pfdone) { R.verdict = dpf::kPfForward; R.acl_over = 0; }
        L.cls = pfw::masq_plan(fc, R, L.m) ? 3u : 2u;
      }
    }
    // the chunk's initial keys; per allocating record the latest earlier one
    // with the same key (pd, in bits 8.. of cls as pd + 1)
    for (int x = lane; x < 256; x += 64) s_hc[wv][x] = 0;
    uint32_t h = 0;
    if (L.cls == 3) {
      h = dpf::fkey_hash(L.m.ik);
      for (int x = 0; x < 11; x++) s_ik[wv][lane][x] = L.m.ik.w[x];
      s_ik[wv][lane][11] = h;
    }
    __syncthreads();
    if (L.cls == 3) atomicAdd(&s_hc[wv][h & 255], 1u);
    __syncthreads();
    const uint64_t c3 = __ballot(L.cls == 3);
    int pd = -1;
    if (L.cls == 3 && s_hc[wv][h & 255] > 1)
      for (int q = lane - 1; q >= 0 && pd < 0; q--) {
        if (!((c3 >> q) & 1) || s_ik[wv][q][11] != h) continue;
        bool eq = true;
        for (int x = 0; x < 11; x++) eq = eq && s_ik[wv][q][x] == L.m.ik.w[x];
        if (eq) pd = q;
      }
    L.cls |= (uint32_t)(pd + 1) << 8;
    // burst-wide: does any initial key repeat (by its hash), does any record run alone
    bool rep = false;
    if ((L.cls & 0xffu) == 3) {
      // (the slot from one hash of the key, the tag from another)
      const uint32_t h2 = dpm::kmix(dpm::kmix(L.m.ik.w[0], L.m.ik.w[1], L.m.ik.w[2]),
                                    dpm::kmix(L.m.ik.w[3], L.m.ik.w[4], L.m.ik.w[5]) ^ L.m.ik.w[6],
                                    dpm::kmix(L.m.ik.w[7], L.m.ik.w[8], L.m.ik.w[9]) ^ L.m.ik.w[10]);
      const unsigned long long want = tag | h2;
      uint32_t x = dpm::kmix(h, 0x5bd1e995u, 0u) & fc.grp_mask;
      for (uint32_t p = 0;; p++) {
        if (p > fc.grp_mask) { rep = true; break; }  // (full: say so)
        const unsigned long long cur = __hip_atomic_load(&fc.dup_tab[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == want) { rep = true; break; }
        if ((cur >> 32) == fc.burst) { x = (x + 1) & fc.grp_mask; continue; }
        const unsigned long long got = atomicCAS(&fc.dup_tab[x], cur, want);
        if (got == cur) break;
        if (got == want) { rep = true; break; }
      }
    }
    pfw::flag_wave(&fc.pf_cnt[28], rep);
    pfw::flag_wave(&fc.pf_cnt[29], (L.cls & 0xffu) == 1);
    // what the lane's bulk serve needs (dp_nat_lane): per 64-record chunk its
    // allocating records (adm[k / 64]; adm is free again once dp_bits_emit has
    // run); burst-wide, the sets they ask (pf_cnt[36] the largest + 1,
    // pf_cnt[37] the complement of the smallest) and whether one's checks fail
    // whatever the tuple or its reverse key may equal its initial key ([38])
    {
      const bool c3 = (L.cls & 0xffu) == 3;
      const uint64_t cm = __ballot(c3);
      if (lane == 0 && b0 + 64 * wv < nl) fc.adm[(b0 >> 6) + wv] = (uint32_t)__popcll(cm);
      pfw::flag_wave(&fc.pf_cnt[38], c3 && (L.m.sfail || L.m.eqp));
      uint32_t hi = c3 ? L.m.set + 1 : 0u, lo = c3 ? ~L.m.set : 0u;
      for (int o = 32; o > 0; o >>= 1) {
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
        lo = max(lo, (uint32_t)__shfl_xor((int)lo, o));
      }
      if (lane == 0 && cm) {
        atomicMax(&fc.pf_cnt[36], hi);
        atomicMax(&fc.pf_cnt[37], lo);
      }
    }
    if (has) {
      const uint4 *w = reinterpret_cast<const uint4 *>(&L);
      for (int x = 0; x < 8; x++) fc.lane_plan[8 * (uint64_t)k + x] = w[x];
      // what the lane's step reads of it (dp_nat_lane): the record, class |
      // (pd + 1) << 8 | eqp << 16 | allow_null << 17, the set and its first
      // region, sfail, the initial key's address words the eqp test compares
      const bool c3r = (L.cls & 0xffu) == 3;
      const uint32_t reg = c3r ? V.setreg()[V.sets()[L.m.set].first_reg] : 0u;
      const uint32_t fl = L.cls | (c3r && L.m.eqp ? 1u << 16 : 0u) | (c3r && L.m.allow_null ? 1u << 17 : 0u);
      fc.lane_key[3 * (uint64_t)k] = make_uint4(L.rec, fl, L.m.set, reg);
      fc.lane_key[3 * (uint64_t)k + 1] = make_uint4(L.m.sfail, L.m.ik.w[7], L.m.ik.w[8], L.m.ik.w[9]);
      fc.lane_key[3 * (uint64_t)k + 2] = make_uint4(L.m.ik.w[10], 0u, 0u, 0u);
    }
    __syncthreads();
  }
}

// The allocating lane is one wave (a 64-work-item workgroup): a wave's memory
// operations are performed in order, so its lanes' stores and later loads
// need wavefront-scope order only -- a compiler barrier, no wait.  (A
// workgroup-scope fence or __syncthreads waits for every store the wave has
// in flight to be acknowledged: ~1 us each, three per block served.)
__device__ __forceinline__ void lane_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
__device__ __forceinline__ void lane_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// dp_nat_lane: the split pass's allocating lane (mode 3), one wave over its
// records in packet order, 64 at a time (dp_nat_lane_plan's chunks).  A
// record whose outcome rests on live flow state (a valid flow with masquerade
// state, the ACL's flow verdict) runs alone, as the one-lane pass runs it.
// The others are decided without the allocator (masq_plan) or allocate; a run
// of them (cut before a record whose initial key an earlier one of the run
// inserts) is served in packet order: where the set's first region's first
// address with free ports has a thread block with free ports, the next
// records of that set take its free ports in order in one step
// (PortAllocator::allocate_port, port_alloc.rs:264-284, record after record:
// a record whose checks fail gives its port back at once, so it takes none),
// else one record allocates alone (a new block, address or region).  The
// block being served stays in LDS from step to step (written back before
// anything else reads the allocator).  Then the run's pairs are created in
// parallel -- or, when no record runs alone and no initial key repeats, every
// pair after the lane (dp_nat_pairs; the allocations go to lane_res).
// The k-th (from 0) set bit of x (k < popc(x))
__device__ __forceinline__ uint32_t nth_bit(uint32_t x, uint32_t k) {
  uint32_t pos = 0;
  for (uint32_t sh = 16; sh; sh >>= 1) {
    const uint32_t c = (uint32_t)__popc(x & ((1u << sh) - 1));
    if (k >= c) { k -= c; x >>= sh; pos += sh; }
  }
  return pos;
}

__global__ void __launch_bounds__(64) dp_nat_lane(const uint8_t *__restrict__ img_base,
                                                  const Image *__restrict__ im, dpf::FlowCtx fc) {
  if (!fc.pf_cnt[1] || !pfw::split_mode(pfw::nat_mode(fc))) return;
  const uint32_t nl = fc.pf_cnt[11];
  const bool post = !fc.pf_cnt[28] && !fc.pf_cnt[29];
  const int t = threadIdx.x;
  const Img g{img_base, *im};
  const pfw::Seq qs{fc, g, false}, qp{fc, g, true};
  const dpm::View V{fc.mq};
  __shared__ uint32_t s_bm[8];  // the block being served: its usage bitmap
  // the block being served: [0] valid, [1] region, [2] address record,
  // [3] block | its first port, [4..7] the address, [8] ports taken since it
  // was loaded, [9] its live ports when loaded
  __shared__ uint32_t s_c[10];
  // the served block's address, as the lane leaves it (every change written
  // through to the allocator as well, never read back while cached): [0]
  // usable blocks, [1] live blocks, [2] not-full blocks, [3] current_alloc_index,
  // [4] the thread block, [5..8] the address (A128), [9] its block flags and
  // order not loaded yet, [10] its record + 1 (0: none); its block flags and
  // block order (bflag, perm)
  __shared__ uint32_t s_a[11];
  __shared__ uint32_t s_flag[64], s_perm[64];
  // the allocator's address records and regions (their offsets read once),
  // and the claims of the region last opened a block in (kClaimsL of them at
  // most; s_cl_n all ones: more, read from the allocator), for block_init
  // (no allocator -- a configuration whose flow-filter rules still ask for
  // masquerade -- and no record here allocates: nothing to read)
  dpm::Addr *const RECS = fc.mq ? V.recs() : nullptr;
  dpm::Region *const REGS = fc.mq ? V.regions() : nullptr;
  constexpr uint32_t kClaimsL = 16;
  __shared__ dpm::Claim s_cl[kClaimsL];
  __shared__ uint32_t s_cl_reg, s_cl_n, s_cl_fam;
  if (t == 0) { s_c[0] = 0; s_a[10] = 0; s_a[9] = 0; s_cl_reg = dpm::kNone; }
  lane_sync();
  // the cached block back to the allocator (by the calling lane); the
  // address's counters stay cached
  auto write_back = [&]() {
    if (s_c[0]) {
      dpm::Addr &A0 = RECS[s_c[2]];
      const uint32_t tb0 = s_c[3] & 0xffu;
      uint32_t full = 0xffffffffu;
      for (int x = 0; x < 8; x++) { A0.bm[tb0][x] = s_bm[x]; full &= s_bm[x]; }
      A0.blive[tb0] = (uint16_t)(s_c[9] + s_c[8]);
      if (full == 0xffffffffu && s_c[8]) A0.nonfull = --s_a[2];
      s_c[0] = 0;
    }
  };
  // the block tb of address a becomes the served one (by the calling lane;
  // the flags and order follow, loaded by the whole wave: s_a[9])
  auto cache_block = [&](uint32_t a, const dpm::Addr &A, uint32_t tb, uint32_t reg, const uint32_t w[4],
                         const dpm::A128 &aa) {
    for (int k = 0; k < 8; k++) s_bm[k] = A.bm[tb][k];
    s_c[0] = 1; s_c[1] = reg; s_c[2] = a; s_c[3] = dpm::block_base(A, tb) | tb;
    for (int k = 0; k < 4; k++) s_c[4 + k] = w[k];
    s_c[8] = 0;
    s_c[9] = A.blive[tb];
    s_a[0] = A.usable; s_a[1] = A.live_blocks; s_a[2] = A.nonfull; s_a[3] = A.cur;
    s_a[4] = (uint32_t)A.thread_block;
    for (int k = 0; k < 4; k++) s_a[5 + k] = aa.w[k];
    s_a[9] = 1;
    s_a[10] = a + 1;
  };
  auto flush = [&]() {
    if (t == 0) { write_back(); s_a[10] = 0; }  // (what runs next changes the allocator itself)
    lane_fence();
    lane_sync();
  };
  // A block of region reg_p to serve (by one lane): the cached one while it
  // has free ports, else (the cached one written back first) the region's
  // first address in use with free ports and its thread block, or for a
  // record that keeps its port (keep: so no block dies on the way) the
  // address's next block, as port_alloc opens it (its thread block full or
  // gone: the first free block from current_alloc_index); anull: the
  // record's allow_null (blocks at port 0 are never opened here)
  auto seek = [&](uint32_t reg_p, bool hit, bool keep, bool anull) {
    if (!hit) {
      write_back();
      s_a[10] = 0;
      const dpm::Region &G = REGS[reg_p];
      uint32_t a = dpm::kNone;
      for (uint32_t x = G.head; x != dpm::kNone; x = RECS[x].next)
        if (dpm::has_free_ports(RECS[x])) { a = x; break; }
      if (a != dpm::kNone && RECS[a].thread_block >= 0) {
        const dpm::Addr &A = RECS[a];
        const uint32_t tb = (uint32_t)A.thread_block;
        if ((A.bflag[tb] & 2) && dpm::block_base(A, tb) != 0) {
          const dpm::A128 aa = dpm::addr_of(V, A);
          uint32_t w[4] = {0, 0, 0, 0};
          if (G.fam == 4) w[0] = aa.w[3];
          else for (int k = 0; k < 4; k++) w[k] = aa.w[k];
          if (pfw::unicast(G.fam, w)) cache_block(a, A, tb, reg_p, w, aa);
        }
      }
    }
    uint32_t fr = 0;
    if (s_c[0])
      for (int k = 0; k < 8; k++) fr += (uint32_t)__popc(~s_bm[k]);
    if (!fr && keep) {
      // the address's next block, as port_alloc opens it (its thread
      // block full or gone: the first free block from
      // current_alloc_index) for a record that keeps its port (so no
      // block dies on the way).  The served block full on an address
      // whose flags are cached: the region's first address with free
      // ports is still that one if it has any (the addresses before
      // it had none, and only this lane allocates), and the next
      // block comes from the cached flags and order
      bool opened = false;
      const uint32_t a0 = s_c[2];
      const bool cached = s_c[0] && s_a[10] == a0 + 1 && !s_a[9];
      write_back();
      if (cached && (s_a[0] > 0 || s_a[2] > 0)) {
        const uint8_t *fl = reinterpret_cast<const uint8_t *>(s_flag);
        const uint8_t *pm = reinterpret_cast<const uint8_t *>(s_perm);
        uint32_t idx = dpm::kNone;
        for (uint32_t k = 0; k < 256; k++) {
          const uint32_t x = (s_a[3] + k) & 0xffu;
          if (fl[x] & 1) { idx = x; break; }
        }
        if (idx != dpm::kNone && pm[idx] != 0) {
          // block_new, from the cache, written through
          dpm::Addr &A = RECS[a0];
          dpm::A128 aa;
          for (int k = 0; k < 4; k++) aa.w[k] = s_a[5 + k];
          const uint32_t base = (uint32_t)pm[idx] << 8;
          uint32_t bm[8];
          if (s_cl_reg != reg_p) {
            const dpm::Region &G = REGS[reg_p];
            const uint32_t n = G.claim_n;
            s_cl_fam = G.fam;
            s_cl_n = n <= kClaimsL ? n : 0xffffffffu;
            const dpm::Claim *C = V.claims() + G.claim_first;
            for (uint32_t c = 0; c < n && c < kClaimsL; c++) s_cl[c] = C[c];
            s_cl_reg = reg_p;
          }
          if (s_cl_n != 0xffffffffu) {
            // dpm::block_init from the claims' copy
            for (int k = 0; k < 8; k++) bm[k] = 0;
            if (!anull && base == 0) bm[0] |= 1u;
            for (uint32_t c = 0; c < s_cl_n; c++) {
              const dpm::Claim &C = s_cl[c];
              if (C.fam != s_cl_fam || !dpm::a_covers(C.net, C.len, C.fam, aa)) continue;
              const uint32_t lo = C.lo > base ? C.lo : base, hi = C.hi < (base | 0xffu) ? C.hi : (base | 0xffu);
              for (uint32_t q = lo; q <= hi && lo <= hi; q++) bm[(q - base) >> 5] |= 1u << ((q - base) & 31);
            }
          } else {
            dpm::block_init(V, REGS[reg_p], aa, base, !anull, bm);
          }
          A.thread_block = (int32_t)idx;
          A.cur = idx;
          A.bflag[idx] = 2;
          A.blive[idx] = 0;
          A.usable = --s_a[0];
          A.live_blocks = ++s_a[1];
          if (!dpm::bm_full(bm)) A.nonfull = ++s_a[2];
          for (int k = 0; k < 8; k++) { A.bm[idx][k] = bm[k]; s_bm[k] = bm[k]; }
          reinterpret_cast<uint8_t *>(s_flag)[idx] = 2;
          s_a[3] = idx;
          s_a[4] = idx;
          s_c[0] = 1; s_c[3] = base | idx; s_c[8] = 0; s_c[9] = 0;
          for (int k = 0; k < 8; k++) fr += (uint32_t)__popc(~bm[k]);
          opened = true;
        }
      }
      if (!opened) {
        s_a[10] = 0;
        const dpm::Region &G = REGS[reg_p];
        uint32_t a = dpm::kNone;
        for (uint32_t x = G.head; x != dpm::kNone; x = RECS[x].next)
          if (dpm::has_free_ports(RECS[x])) { a = x; break; }
        if (a != dpm::kNone) {
          dpm::Addr &A = RECS[a];
          const int32_t tb = A.thread_block;
          const bool spent = tb < 0 || !(A.bflag[tb] & 2) || dpm::bm_full(A.bm[tb]);
          uint32_t idx = dpm::kNone;
          if (spent)
            for (uint32_t k = 0; k < 256; k++) {
              const uint32_t x = (A.cur + k) & 0xffu;
              if (A.bflag[x] & 1) { idx = x; break; }
            }
          const dpm::A128 aa = dpm::addr_of(V, A);
          uint32_t w[4] = {0, 0, 0, 0};
          if (G.fam == 4) w[0] = aa.w[3];
          else for (int k = 0; k < 4; k++) w[k] = aa.w[k];
          if (idx != dpm::kNone && dpm::block_base(A, idx) != 0 && pfw::unicast(G.fam, w)) {
            A.thread_block = (int32_t)idx;
            A.cur = idx;
            dpm::block_new(V, a, idx, anull);
            cache_block(a, A, idx, reg_p, w, aa);
          }
        }
      }
    }
  };
  // then, by the wave: a newly cached address's block flags and order
  auto seek_flags = [&]() {
    lane_sync();
    if (s_a[9] && s_c[0]) {
      const dpm::Addr &A = RECS[s_c[2]];
      s_flag[t] = reinterpret_cast<const uint32_t *>(A.bflag)[t];
      s_perm[t] = reinterpret_cast<const uint32_t *>(A.perm)[t];
      lane_sync();
      if (t == 0) s_a[9] = 0;
      lane_sync();
    }
  };
  // seek's common case for the bulk serve, by the whole wave: the served
  // block full, the address's block flags and the region's claims cached --
  // the block written back and the address's next block opened from the
  // cache (the first free block from current_alloc_index, its bitmap a word
  // per lane), as seek's cached path does.  false: nothing done (seek runs).
  auto open_next = [&](uint32_t reg) -> bool {
    if (!s_c[0] || s_c[1] != reg || s_a[10] != s_c[2] + 1 || s_a[9]) return false;
    if (s_cl_reg != reg || s_cl_n == 0xffffffffu) return false;
    const uint32_t a0 = s_c[2], tb0 = s_c[3] & 0xffu, taken = s_c[8];
    // (the served block is full: its write-back drops the not-full count
    // when this visit filled it)
    const uint32_t nf = s_a[2] - (taken ? 1u : 0u);
    if (!(s_a[0] > 0 || nf > 0)) return false;
    const uint8_t *fl = reinterpret_cast<const uint8_t *>(s_flag);
    const uint8_t *pm = reinterpret_cast<const uint8_t *>(s_perm);
    const uint32_t cur = s_a[3];
    uint32_t idx = dpm::kNone;
    for (uint32_t k0 = 0; k0 < 256 && idx == dpm::kNone; k0 += 64) {
      const uint64_t m = __ballot(fl[(cur + k0 + t) & 0xffu] & 1);
      if (m) idx = (cur + k0 + (uint32_t)__ffsll((long long)m) - 1) & 0xffu;
    }
    if (idx == dpm::kNone || pm[idx] == 0) return false;
    const uint32_t base = (uint32_t)pm[idx] << 8;
    // the new block's bitmap (dpm::block_init: the claims covering the
    // address; base != 0, so no null port), word t on lane t < 8
    uint32_t w = 0;
    if (t < 8) {
      dpm::A128 aa;
      for (int k = 0; k < 4; k++) aa.w[k] = s_a[5 + k];
      const uint32_t wlo = base + 32u * t, whi = wlo + 31u;
      for (uint32_t c = 0; c < s_cl_n; c++) {
        const dpm::Claim &C = s_cl[c];
        if (C.fam != s_cl_fam || !dpm::a_covers(C.net, C.len, C.fam, aa)) continue;
        const uint32_t lo = C.lo > wlo ? C.lo : wlo, hi = C.hi < whi ? C.hi : whi;
        if (lo <= hi) {
          const uint32_t nb = hi - lo + 1;
          w |= (nb == 32 ? 0xffffffffu : ((1u << nb) - 1u)) << (lo - wlo);
        }
      }
    }
    const bool full = __ballot(t < 8 && w == 0xffffffffu) == 0xffull;
    dpm::Addr &A = RECS[a0];
    if (t < 8) {
      A.bm[tb0][t] = s_bm[t];  // (write_back)
      A.bm[idx][t] = w;
    }
    if (t == 0) {
      A.blive[tb0] = (uint16_t)(s_c[9] + taken);
      A.thread_block = (int32_t)idx;
      A.cur = idx;
      A.bflag[idx] = 2;
      A.blive[idx] = 0;
      A.usable = s_a[0] - 1;
      A.live_blocks = s_a[1] + 1;
      if (!full) A.nonfull = nf + 1;
      else if (taken) A.nonfull = nf;
    }
    lane_sync();
    if (t < 8) s_bm[t] = w;
    if (t == 0) {
      s_a[0] -= 1;
      s_a[1] += 1;
      s_a[2] = full ? nf : nf + 1;
      reinterpret_cast<uint8_t *>(s_flag)[idx] = 2;
      s_a[3] = idx;
      s_a[4] = idx;
      s_c[0] = 1; s_c[3] = base | idx; s_c[8] = 0; s_c[9] = 0;
    }
    lane_sync();
    return true;
  };
  // a record's full plan (the allocation alone, the pairs in the lane)
  auto plan_of = [&](uint32_t k) {
    pfw::LanePlan P;
    uint4 *w = reinterpret_cast<uint4 *>(&P);
    for (int j = 0; j < 8; j++) w[j] = fc.lane_plan[8 * (uint64_t)k + j];
    return P;
  };
  // what a step needs of the chunk's records (dp_nat_lane_plan's lane_key),
  // the next chunk's loaded while this one is served
  auto key_of = [&](uint32_t k0, uint4 &a, uint4 &b, uint4 &c) {
    if (k0 + t < nl) {
      const uint64_t k = 3 * (uint64_t)(k0 + t);
      a = fc.lane_key[k]; b = fc.lane_key[k + 1]; c = fc.lane_key[k + 2];
    } else {
      a = b = c = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  uint32_t fast_n = 0, lone_n = 0, solo_n = 0;
  // where the lane's time goes (clock64 ticks: chunk keys, allocations, pairs,
  // records alone, the step's block, the batch served, allocations alone),
  // for the counters [19..25] in units of 1024 ticks
  uint64_t tk[7] = {0, 0, 0, 0, 0, 0, 0}, t0 = clock64(), ta;
  uint32_t steps = 0;
  // The bulk serve (post: no record alone, no initial key repeated; every
  // allocating record of one set, none whose checks fail whatever the tuple
  // or whose reverse key may equal its initial key).  Then the steps below
  // hand the allocating records the set's first region's ports in packet
  // order whatever the records are: the served block's lowest free ports
  // first, block after block as they open them.  So the wave walks the blocks
  // alone, logging per block its free ports and the allocation ranks it
  // serves (adm: the chunks' allocating records, made a prefix, then the
  // log), and dp_nat_lane_assign gives each record its port in parallel.
  // Where no block is to be had that way, the record of the next rank
  // allocates alone, as the steps would (a one-rank entry, or one without a
  // port); with the log full, the steps take over from that record.
  uint32_t kstart = 0;
  if (post && fc.force_seq != 2 && fc.force_seq != 5 && !fc.pf_cnt[38] &&
      (!fc.pf_cnt[36] || ~fc.pf_cnt[37] + 1u == fc.pf_cnt[36])) {
    const uint32_t nch = (nl + 63) / 64;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
      const uint32_t v = c0 + t < nch ? fc.adm[c0 + t] : 0u;
      uint32_t x = v;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (t >= o) x += y;
      }
      if (c0 + t < nch) fc.adm[c0 + t] = carry + x - v;
      carry += (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    }
    const uint32_t total = carry;
    if (t == 0) fc.adm[nch] = total;
    lane_fence();
    lane_sync();
    // the lane record of allocation rank r < total: in the last chunk whose
    // prefix is at most r (adm[nch] = total), by the wave
    auto rank_rec = [&](uint32_t r) {
      uint32_t lo = 0, hi = nch;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (fc.adm[mid] <= r) lo = mid;
        else hi = mid;
      }
      const uint32_t k = 64 * lo + t;
      const bool c3 = k < nl && (fc.lane_key[3 * (uint64_t)k].y & 0xffu) == 3;
      const uint64_t cm = __ballot(c3);
      const uint32_t j = r - fc.adm[lo], lo32 = (uint32_t)__popc((uint32_t)cm);
      return 64 * lo + (j < lo32 ? nth_bit((uint32_t)cm, j) : 32 + nth_bit((uint32_t)(cm >> 32), j - lo32));
    };
    const uint32_t off = (nch + 1 + 15) & ~15u;
    const uint32_t cap = fc.n + 1 > off ? (fc.n + 1 - off) / 16 : 0u;
    uint32_t *blog = fc.adm + off;
    uint32_t served = 0, ents = 0;
    if (total) {
      const uint32_t reg = V.setreg()[V.sets()[fc.pf_cnt[36] - 1].first_reg];
      while (served < total && ents < cap) {
        ta = clock64();
        uint32_t f = 0;
        const bool hit = s_c[0] && s_c[1] == reg;
        if (hit && t < 8) f = ~s_bm[t];
        if (!hit || !__ballot(f != 0)) {
          if (!(hit && fc.force_seq != 6 && open_next(reg))) {
            if (t == 0) seek(reg, hit, true, false);
            seek_flags();
          }
          f = s_c[0] && s_c[1] == reg && t < 8 ? ~s_bm[t] : 0u;
        }
        const uint32_t fc_n = (uint32_t)__popc(f);
        uint32_t pre = fc_n;
        for (int o = 1; o < 8; o <<= 1) {
          const uint32_t v = (uint32_t)__shfl_up((int)pre, o);
          if (t >= o) pre += v;
        }
        const uint32_t fr = (uint32_t)__builtin_amdgcn_readlane((int)pre, 7);
        { const uint64_t x = clock64(); tk[4] += x - ta; ta = x; }
        uint32_t *e = blog + 16 * (uint64_t)ents;
        if (!fr) {
          // alone, as resolve_masq allocates (on the allocator as it is): the
          // entry's base all ones when the record gets no port
          const uint32_t k = rank_rec(served);
          flush();
          if (t == 0) {
            const pfw::LanePlan P = plan_of(k);
            dpf::PfReq &Rk = fc.pf[P.rec];
            uint32_t rec = 0, aport = 0, aip[4] = {0, 0, 0, 0};
            bool got = false;
            const uint32_t er = dpm::set_alloc(V, P.m.set, P.m.allow_null, rec, aport);
            if (er != dpm::OK) {
              Rk.mverdict = pfw::masq_done(er);
            } else {
              pfw::masq_aip(fc, Rk, rec, aip);
              const uint32_t v = pfw::masq_post(Rk, P.m, aip, aport);
              if (v) { dpm::release(V, rec, aport); Rk.mverdict = v; }
              else got = true;
            }
            e[0] = served; e[1] = 1; e[2] = rec; e[3] = got ? aport & ~0xffu : 0xffffffffu;
            for (int x = 0; x < 4; x++) e[4 + x] = aip[x];
            for (int x = 0; x < 8; x++) e[8 + x] = got && x == (int)((aport & 0xffu) >> 5) ? 1u << (aport & 31) : 0u;
            lone_n++;
          }
          lane_fence();
          lane_sync();
          served++;
          ents++;
          { const uint64_t x = clock64(); tk[6] += x - ta; ta = x; }
          continue;
        }
        const uint32_t taken = total - served < fr ? total - served : fr;
        // the log entry: first rank, ranks served, address record, block
        // base, the address, the block's free ports before
        const uint32_t fw = (uint32_t)__shfl((int)f, t & 7);
        uint32_t ev = 0;
        if (t == 0) ev = served;
        else if (t == 1) ev = taken;
        else if (t == 2) ev = s_c[2];
        else if (t == 3) ev = s_c[3] & ~0xffu;
        else if (t < 8) ev = s_c[t];
        else ev = fw;
        if (t < 16) e[t] = ev;
        // the block's bitmap after `taken` allocations: its lowest free ports
        if (t < 8) {
          const uint32_t below = pre - fc_n;
          const uint32_t n = taken > below ? (taken - below < fc_n ? taken - below : fc_n) : 0u;
          if (n) s_bm[t] = ~f | (n == fc_n ? f : f & ((1u << nth_bit(f, n)) - 1));
        }
        if (t == 0) { s_c[8] += taken; fast_n += taken; }
        served += taken;
        ents++;
        steps++;
        lane_sync();
        { const uint64_t x = clock64(); tk[5] += x - ta; ta = x; }
      }
    }
    // the steps below start at the record of rank `served` (the log full)
    kstart = served < total ? rank_rec(served) : nl;
    if (t == 0) {
      fc.pf_cnt[35] = kstart;
      fc.pf_cnt[39] = ents;
    }
    t0 = clock64();
  }
  uint4 N0, N1, N2;
  key_of(kstart, N0, N1, N2);
  for (uint32_t k0 = kstart; k0 < nl; k0 += 64) {
    const uint32_t cnt = nl - k0 < 64 ? nl - k0 : 64;
    const uint4 K0 = N0, K1 = N1, K2 = N2;
    if (k0 + 64 < nl) key_of(k0 + 64, N0, N1, N2);
    // the record's class (1 alone, 2 decided, 3 allocates), the latest earlier
    // record of the chunk with its initial key, its set and that set's first
    // region, the verdict its checks give whatever the tuple, its address
    const uint32_t ri = K0.x, cls = K0.y & 0xffu;
    const int pd = (int)((K0.y >> 8) & 0xffu) - 1;
    const bool eqp = (K0.y >> 16) & 1u;
    const uint32_t mset = K0.z, mreg = K0.w, sfail = K1.x;
    const uint32_t ia[4] = {K1.y, K1.z, K1.w, K2.x};
    dpf::PfReq &R = fc.pf[ri];
    const uint64_t c1 = __ballot(cls == 1), c3 = __ballot(cls == 3);
    const uint64_t cuts = __ballot(cls == 1 || (cls == 3 && pd >= 0));
    { const uint64_t x = clock64(); tk[0] += x - t0; t0 = x; }
    // the lane's allocation: ok (a pair to create), else its verdict is set
    bool ok = false, done = cls != 3;
    uint32_t rec = 0, aport = 0, aip[4] = {0, 0, 0, 0};
    uint32_t i = 0;
    while (i < cnt) {
      if ((c1 >> i) & 1) {
        flush();
        if (t == (int)i) {
          if (R.bits & dpf::kPqPfDone) {
            R.mverdict = dpf::kPfForward;
            pfw::resolve_masq(qs, R);
          } else {
            pfw::resolve_one(qs, R);
          }
          solo_n++;
        }
        lane_fence();
        { const uint64_t x = clock64(); tk[3] += x - t0; t0 = x; }
        i++;
        continue;
      }
      // the run [i, j): up to the next record alone, or one whose initial
      // key an earlier record of the run inserts (candidates: cuts)
      uint32_t j = cnt;
      for (uint64_t c = cuts & ~((2ull << i) - 1); c; c &= c - 1) {
        const uint32_t q = (uint32_t)__ffsll((long long)c) - 1;
        if (q >= cnt) break;
        if (((c1 >> q) & 1) || (int)__shfl(pd, (int)q) >= (int)i) { j = q; break; }
      }
      const uint64_t run = (j == 64 ? ~0ull : ((1ull << j) - 1)) & ~((1ull << i) - 1);
      // the run's allocations, in packet order
      for (;;) {
        const uint64_t pend = __ballot(!done) & c3 & run;
        if (!pend) break;
        const int p = __ffsll((long long)pend) - 1;
        const uint32_t set_p = (uint32_t)__shfl((int)mset, p), reg_p = (uint32_t)__shfl((int)mreg, p);
        ta = clock64();
        steps++;
        // the set's first region's block being served: the cached one while
        // it has free ports, else (the cached one written back first) the
        // region's first address in use with free ports and its thread block,
        // or for a record that keeps its port (so no block dies on the way)
        // the address's next block, as port_alloc opens it (its thread block
        // full or gone: the first free block from current_alloc_index)
        uint32_t f = 0;
        const bool hit = s_c[0] && s_c[1] == reg_p;
        if (hit && t < 8) f = ~s_bm[t];
        if ((!hit || !__ballot(f != 0)) && fc.force_seq != 2) {
          if (t == p) seek(reg_p, hit, !sfail, (K0.y >> 17) & 1u);
          seek_flags();
          f = s_c[0] && s_c[1] == reg_p && t < 8 ? ~s_bm[t] : 0u;
        }
        // the block's free ports: per word (lanes 0..7) and before it
        const uint32_t fc_n = (uint32_t)__popc(f);
        uint32_t pre = fc_n;
        for (int o = 1; o < 8; o <<= 1) {
          const uint32_t v = (uint32_t)__shfl_up((int)pre, o);
          if (t >= o) pre += v;
        }
        const uint32_t fr_all = (uint32_t)__builtin_amdgcn_readlane((int)pre, 7);
        // a record whose reverse key could equal its initial key (related_pair)
        // at the block's address goes alone, and stops the batch before it
        bool eqa = eqp;
        for (int k = 0; k < 4; k++) eqa = eqa && ia[k] == pfw::bswap(s_c[4 + k]);
        const bool p_eq = (__ballot(eqa) >> p) & 1;
        const uint32_t fr = fr_all && !p_eq ? fr_all : 0u;
        { const uint64_t x = clock64(); tk[4] += x - ta; ta = x; }
        if (fr) {
          // the records from p on asking the same set, up to one whose
          // reverse key could equal its initial key: served while the block
          // has free ports, in packet order
          const uint32_t a = s_c[2], base = s_c[3] & ~0xffu;
          bool stop = false;
          if (!done && ((pend >> t) & 1)) stop = mset != set_p || eqa;
          const uint64_t st = __ballot(stop) & pend;
          const uint64_t grp = st ? pend & ((1ull << (__ffsll((long long)st) - 1)) - 1) : pend;
          const bool mine = (grp >> t) & 1;
          const uint64_t cons = __ballot(mine && !sfail) & grp;
          const uint32_t before = (uint32_t)__popcll(cons & lanes_below(t));
          const bool served = mine && before < fr;
          const uint32_t taken = (uint32_t)__popcll(cons) < fr ? (uint32_t)__popcll(cons) : fr;
          // the before-th free port: its word, then its bit
          uint32_t wsel = 0;
          for (int x = 0; x < 7; x++) wsel += (uint32_t)__builtin_amdgcn_readlane((int)pre, x) <= before ? 1u : 0u;
          const uint32_t fw = (uint32_t)__shfl((int)f, (int)wsel), fb = (uint32_t)__shfl((int)(pre - fc_n), (int)wsel);
          if (served) {
            if (sfail) {
              R.mverdict = sfail;
            } else {
              rec = a;
              aport = base + 32 * wsel + nth_bit(fw, before - fb);
              for (int x = 0; x < 4; x++) aip[x] = s_c[4 + x];
              ok = true;
            }
            done = true;
          }
          // the block's bitmap after `taken` allocations: its lowest free ports
          if (t < 8) {
            const uint32_t below = pre - fc_n;
            const uint32_t n = taken > below ? (taken - below < fc_n ? taken - below : fc_n) : 0u;
            if (n) s_bm[t] = ~f | (n == fc_n ? f : f & ((1u << nth_bit(f, n)) - 1));
          }
          if (t == 0) s_c[8] += taken;
          if (t == p) fast_n += taken;
          lane_sync();
          { const uint64_t x = clock64(); tk[5] += x - ta; ta = x; }
        } else {
          // alone, as resolve_masq allocates (on the allocator as it is)
          flush();
          if (t == p) {
            const pfw::LanePlan P = plan_of(k0 + p);
            const uint32_t e = dpm::set_alloc(V, P.m.set, P.m.allow_null, rec, aport);
            if (e != dpm::OK) {
              R.mverdict = pfw::masq_done(e);
            } else {
              pfw::masq_aip(fc, R, rec, aip);
              const uint32_t v = pfw::masq_post(R, P.m, aip, aport);
              if (v) { dpm::release(V, rec, aport); R.mverdict = v; }
              else ok = true;
            }
            done = true;
            lone_n++;
          }
          lane_fence();
          lane_sync();
          { const uint64_t x = clock64(); tk[6] += x - ta; ta = x; }
        }
      }
      { const uint64_t x = clock64(); tk[1] += x - t0; t0 = x; }
      if (post) {
        // the allocation, for dp_nat_pairs
        if ((run >> t) & 1)
          fc.lane_res[2 * (uint64_t)(k0 + t)] = make_uint4(ok ? 1u : 0u, rec, aport, 0u),
          fc.lane_res[2 * (uint64_t)(k0 + t) + 1] = make_uint4(aip[0], aip[1], aip[2], aip[3]);
        ok = false;
      } else {
        // the run's pairs, in parallel (distinct initial keys; distinct tuples)
        bool give_back = false;
        if (ok && ((run >> t) & 1)) {
          const pfw::LanePlan P = plan_of(k0 + t);
          if (!pfw::masq_pair(qp, R, P.m, rec, aport, aip, give_back)) atomicAdd(&fc.pf_cnt[16], 1u);
          ok = false;
        }
        lane_fence();
        if (__ballot(give_back)) {
          flush();
          for (uint64_t gb = __ballot(give_back); gb; gb &= gb - 1) {
            if (t == __ffsll((long long)gb) - 1) dpm::release(V, rec, aport);
            lane_fence();
          }
        }
      }
      { const uint64_t x = clock64(); tk[2] += x - t0; t0 = x; }
      i = j;
    }
  }
  flush();
  if (t == 0 && !post) {
    // the flows replaced during the burst are dropped after it, with the
    // allocations their masquerade state owns
    for (uint32_t k = 0; k < fc.pf_cnt[3]; k++) dpm::release(V, fc.mq_rel[2 * k], fc.mq_rel[2 * k + 1]);
  }
  uint32_t ln = lone_n, fn = fast_n, sn = solo_n;
  for (int o = 32; o > 0; o >>= 1) { ln += __shfl_xor(ln, o); fn += __shfl_xor(fn, o); sn += __shfl_xor(sn, o); }
  if (t == 0) {
    fc.pf_cnt[14] += fn;
    fc.pf_cnt[18] += sn;
    for (int k = 0; k < 7; k++) fc.pf_cnt[19 + k] = (uint32_t)(tk[k] >> 10);
    fc.pf_cnt[26] = steps;
  }
  uint32_t v = qp.added;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (t == 0) {
    fc.pf_cnt[15] += ln;
    if (v) atomicAdd(reinterpret_cast<unsigned long long *>(&fc.tmeta[2]), (unsigned long long)v);
  }
}

// dp_nat_lane_assign: the lane's bulk-served records (lane records before
// pf_cnt[35], dp_nat_lane) their allocations for dp_nat_pairs, in parallel:
// an allocating record's rank (its chunk's prefix in adm, plus those before it
// in the chunk) names the logged block serving it and its free port there --
// the ranks a block serves take its lowest free ports in order.
__global__ void __launch_bounds__(256) dp_nat_lane_assign(dpf::FlowCtx fc) {
  if (!fc.pf_cnt[1] || !pfw::split_mode(pfw::nat_mode(fc))) return;
  const uint32_t kend = fc.pf_cnt[35];
  if (!kend) return;
  const uint32_t nl = fc.pf_cnt[11], nch = (nl + 63) / 64, ents = fc.pf_cnt[39];
  const uint32_t *blog = fc.adm + ((nch + 1 + 15) & ~15u);
  const int lane = threadIdx.x & 63;
  for (uint32_t b0 = blockIdx.x * 256; b0 < kend; b0 += gridDim.x * 256) {  // (uniform per block)
    const uint32_t k = b0 + (threadIdx.x & ~63u) + lane;  // (a wave: one 64-record chunk)
    const bool has = k < kend;
    const uint32_t cls = has ? fc.lane_key[3 * (uint64_t)k].y & 0xffu : 0u;
    const uint64_t cm = __ballot(cls == 3);
    uint4 r0 = make_uint4(0u, 0u, 0u, 0u), r1 = r0;
    if (cls == 3) {
      const uint32_t rank = fc.adm[k >> 6] + (uint32_t)__popcll(cm & lanes_below(lane));
      uint32_t lo = 0, hi = ents;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (blog[16 * (uint64_t)mid] <= rank) lo = mid;
        else hi = mid;
      }
      const uint32_t *e = blog + 16 * (uint64_t)lo;
      if (e[3] != 0xffffffffu) {  // (else an allocation alone that got no port)
        uint32_t j = rank - e[0], port = 0;
        for (int w = 0; w < 8; w++) {
          const uint32_t f = e[8 + w], c = (uint32_t)__popc(f);
          if (j < c) { port = e[3] + 32 * w + nth_bit(f, j); break; }
          j -= c;
        }
        r0 = make_uint4(1u, e[2], port, 0u);
        r1 = make_uint4(e[4], e[5], e[6], e[7]);
      }
    }
    if (has) {
      fc.lane_res[2 * (uint64_t)k] = r0;
      fc.lane_res[2 * (uint64_t)k + 1] = r1;
    }
  }
}

// dp_nat_pairs: the allocating lane's pairs, all at once, when no record of
// it ran alone and no initial key repeats (dp_nat_lane_plan): then no pair's
// inserts meet another's keys or any record's live flow state, and the lane's
// allocations never depended on them (the table has room: no insert is
// refused).  dp_nat_lane_end then drops the replaced fills' allocations.
__global__ void __launch_bounds__(256) dp_nat_pairs(const uint8_t *__restrict__ img_base,
                                                    const Image *__restrict__ im, dpf::FlowCtx fc) {
  if (!fc.pf_cnt[1] || !pfw::split_mode(pfw::nat_mode(fc)) || fc.pf_cnt[28] || fc.pf_cnt[29]) return;
  const uint32_t nl = fc.pf_cnt[11];
  const Img g{img_base, *im};
  const pfw::Seq qp{fc, g, true};
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < nl; k += gridDim.x * 256) {
    const uint4 r0 = fc.lane_res[2 * (uint64_t)k];
    if (!r0.x) continue;
    const uint4 r1 = fc.lane_res[2 * (uint64_t)k + 1];
    pfw::LanePlan P;
    uint4 *w = reinterpret_cast<uint4 *>(&P);
    for (int j = 0; j < 8; j++) w[j] = fc.lane_plan[8 * (uint64_t)k + j];
    const uint32_t aip[4] = {r1.x, r1.y, r1.z, r1.w};
    bool give_back = false;
    if (!pfw::masq_pair(qp, fc.pf[P.rec], P.m, r0.y, r0.z, aip, give_back)) atomicAdd(&fc.pf_cnt[16], 1u);
  }
  uint32_t v = qp.added;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0 && v)
    atomicAdd(reinterpret_cast<unsigned long long *>(&fc.tmeta[2]), (unsigned long long)v);
}
// (also after the connection-parallel port-forwarding pass, modes 2 and 4:
// a creation there may replace a masqueraded flow, whose allocation then goes
// when the burst ends, as in the one-lane pass)
__global__ void dp_nat_lane_end(dpf::FlowCtx fc) {
  if (!fc.pf_cnt[1] || !fc.mq || !fc.pf_cnt[3]) return;
  const uint32_t mode = pfw::nat_mode(fc);
  if (mode == 1 || (pfw::split_mode(mode) && (fc.pf_cnt[28] || fc.pf_cnt[29]))) return;
  const dpm::View V{fc.mq};
  for (uint32_t k = 0; k < fc.pf_cnt[3]; k++) dpm::release(V, fc.mq_rel[2 * k], fc.mq_rel[2 * k + 1]);
}

// dp_acl_classify: AclFilter's classification alone (dpgpu.h "The ACL
// classifier alone"), one key per work-item: the peering's ACL group, its
// first matching rule, else the peering default, else Allow -- stage_acl's
// decision without a packet around it.
__global__ void __launch_bounds__(256) dp_acl_classify_k(const uint8_t *__restrict__ img_base,
                                                         const Image *__restrict__ im,
                                                         const dp_acl_key_t *__restrict__ keys,
                                                         dp_acl_result_t *__restrict__ out, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const dp_acl_key_t k = keys[i];
  dp_acl_result_t r{};
  r.rule = 0xffffffffu;
  if (k.family != 4 && k.family != 6) { out[i] = r; return; }
  const Img g{img_base, *im};
  const int t = k.family == 4 ? 0 : 1;
  auto be = [&](const uint8_t *a, int o) {
    return ((uint32_t)a[o] << 24) | ((uint32_t)a[o + 1] << 16) | ((uint32_t)a[o + 2] << 8) | a[o + 3];
  };
  Key128 ks, kd;
  if (t == 0) {
    ks = Key128{0, be(k.src, 0)};
    kd = Key128{0, be(k.dst, 0)};
  } else {
    ks = Key128{((uint64_t)be(k.src, 0) << 32) | be(k.src, 4), ((uint64_t)be(k.src, 8) << 32) | be(k.src, 12)};
    kd = Key128{((uint64_t)be(k.dst, 0) << 32) | be(k.dst, 4), ((uint64_t)be(k.dst, 8) << 32) | be(k.dst, 12)};
  }
  int32_t ag = -1;
  uint32_t def = 0, pi;
  if (hash_find(g, g.im.pairs, k.src_vni, k.dst_vni, 0, pi)) {
    const PairRec &P = g.at<PairRec>(g.im.pair_recs)[pi];
    ag = P.acl[t];
    def = P.acl_def;
  }
  const Hit h = classify<W_ACTION | W_ORIG>(g, CLS_ARRAYS(acl, t), ag, t, k.proto, ks, kd, k.sport, k.dport);
  if (h.rule >= 0) {
    r.rule = h.orig;
    r.action = (uint8_t)(h.action & 0xffu);
    r.scope = (uint8_t)(h.action >> 8);
    r.acl = r.action == DP_ACL_DENY ? 2 : 1;
  } else if (def) {
    r.action = (uint8_t)(def - 1);
    r.acl = r.action == DP_ACL_DENY ? 4 : 3;
  } else {
    r.action = DP_ACL_ALLOW;
    r.acl = 5;
  }
  out[i] = r;
}

// dp_ff_classify: FlowFilterContext::lookup_batch alone (dpgpu.h "The
// flow-filter classifier alone"), one input per work-item -- stage_flow_filter's
// two lookups without a packet around them: stage 1 over the (src VNI,
// GateVni) group of the remote rules, on a hit stage 2 over the (src VNI,
// verdict VPC, SourceGate) group of the local rules (flow-filter/src/context/
// tables.rs:854-915).  stage: 0 both (lookup_batch), 1 the remote rules alone,
// 2 the local rules alone (dst_vni is then the local key's VPC).
__global__ void __launch_bounds__(256) dp_ff_classify_k(const uint8_t *__restrict__ img_base,
                                                        const Image *__restrict__ im,
                                                        const dp_ff_input_t *__restrict__ in,
                                                        dp_ff_result_t *__restrict__ out, uint32_t n, int stage) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const dp_ff_input_t q = in[i];
  dp_ff_result_t r{};
  r.outcome = stage == 2 ? DP_FF_SOURCE_MISS : DP_FF_DESTINATION_MISS;
  if (q.src_family != q.dst_family || (q.src_family != 4 && q.src_family != 6)) { out[i] = r; return; }
  const Img g{img_base, *im};
  const int t = q.src_family == 4 ? 0 : 1;
  auto be = [&](const uint8_t *a, int o) {
    return ((uint32_t)a[o] << 24) | ((uint32_t)a[o + 1] << 16) | ((uint32_t)a[o + 2] << 8) | a[o + 3];
  };
  auto key = [&](const uint8_t *a) {
    return t == 0 ? Key128{0, be(a, 0)}
                  : Key128{((uint64_t)be(a, 0) << 32) | be(a, 4), ((uint64_t)be(a, 8) << 32) | be(a, 12)};
  };
  uint32_t gi, dvni = q.dst_vni;
  if (stage != 2) {
    const int32_t rg = hash_find(g, g.im.ff_remote[t].groups, q.src_vni, q.dst_vni, 0, gi) ? (int32_t)gi : -1;
    const Hit rh = classify<W_ACTION | W_ACTION2>(g, CLS_ARRAYS(ff_remote, t), rg, t, q.proto, Key128{0, 0},
                                                  key(q.dst), 0, q.dport);
    if (rh.rule < 0) { out[i] = r; return; }
    r.dst_vni = rh.action;
    r.dst_nat = (uint8_t)rh.action2;
    dvni = rh.action;
    r.outcome = stage == 1 ? DP_FF_ROUTE : DP_FF_SOURCE_MISS;
    if (stage == 1) { out[i] = r; return; }
  }
  const int32_t lg = hash_find(g, g.im.ff_local[t].groups, q.src_vni, dvni, q.gate, gi) ? (int32_t)gi : -1;
  const Hit lh = classify<W_ACTION>(g, CLS_ARRAYS(ff_local, t), lg, t, q.proto, key(q.src), Key128{0, 0},
                                    q.sport, 0);
  if (lh.rule >= 0) {
    r.src_nat = (uint8_t)lh.action;
    r.outcome = DP_FF_ROUTE;
  }
  out[i] = r;
}

// After the burst's pipeline kernel (flows variant), on its stream.
// dp_flow_fixup: a verdict "allowed as the reply of a flow-scope-allowed
// flow" stands only if the flow pair was still valid when the packet reached
// the ACL: not invalidated by the flow filter (mark 0: the flow filter runs
// over the whole burst before any ACL) nor by the deny of an earlier packet
// (mark idx + 1).  Otherwise the peering default applies; a default Deny
// drops the packet at the ACL with its metadata as it stood there.
__global__ void __launch_bounds__(256) dp_flow_fixup(const uint8_t *__restrict__ img_base,
                                                     const Image *__restrict__ im, dpf::FlowCtx fc,
                                                     const dp_pkt_in_t *__restrict__ in,
                                                     dp_pkt_out_t *__restrict__ out,
                                                     dp_pkt_meta_t *__restrict__ meta,
                                                     unsigned long long *__restrict__ stats) {
  const uint32_t cnt = fc.sens[0];
  const dpf::SensRec *recs = reinterpret_cast<const dpf::SensRec *>(fc.sens + 8);
  const uint32_t nrep = fc.pf_cnt[2];
  // a fill for packet idx: 1 in the table (its burst-local mark), 0 not in
  // the table as the burst started, -1 replaced by the NAT pass before idx
  // (a fill replaced by packet j > idx counts with the mark it had); the
  // replaced fills by their keyed index
  auto fill_at = [&](uint32_t sl, uint32_t tag, uint32_t idx, uint32_t &mark) -> int {
    if (sl > fc.mask) return 0;
    if (fc.slots[sl].state == tag) { mark = fc.slots[sl].mark; return 1; }
    if (!nrep) return 0;
    uint32_t h = dpf::repl_hash(sl, tag) & fc.rmask;
    for (uint32_t p = 0; p <= fc.rmask; p++, h = (h + 1) & fc.rmask) {
      const uint4 e = fc.repl[h];
      if (e.y != fc.burst) return 0;
      if (e.x == sl && e.z == tag) {
        mark = fc.pf_repl[4 * e.w + 3];
        return fc.pf_repl[4 * e.w + 2] > idx ? 1 : -1;
      }
    }
    return 0;
  };
  for (uint32_t r = blockIdx.x * 256 + threadIdx.x; r < cnt; r += gridDim.x * 256) {
    const dpf::SensRec R = recs[r];
    // the pair is invalid if either flow was invalidated (invalidate_pair
    // marks the flow it was called on; the related flow only while alive)
    uint32_t ms = 0, mr = dpf::kIdleMark;
    const int own = fill_at(R.slot, R.slot_tag, R.idx, ms);
    const int rel = fill_at(R.related, R.related_tag, R.idx, mr);
    if (own == 1 && ms > R.idx && rel >= 0 && (rel == 0 || mr > R.idx)) continue;  // still valid
    dp_pkt_out_t o = out[R.idx];
    o.acl = (uint8_t)R.def_acl;
    if (meta) meta[R.idx].acl_rule = 0xffffffffu;
    if (R.def_acl == 4) {
      if (stats && o.done < DP_DONE_COUNT) {
        atomicAdd(&stats[o.done], ~0ull);  // -1
        atomicAdd(&stats[DP_DONE_ACL_DROPPED], 1ull);
      }
      o.done = DP_DONE_ACL_DROPPED;
      o.off = in[R.idx].off;
      o.len = in[R.idx].len;
      o.meta_flags = (uint16_t)R.meta_flags;
      o.oif = R.oif;
      if (meta) {
        // PacketMeta as it stood at the ACL
        dp_pkt_meta_t m = meta[R.idx];
        m.fib_entry = R.fib_entry;
        m.dst_vni = R.dst_vni;
        m.pm_flags &= (uint8_t)~(DP_PM_HAS_VRF | DP_PM_HAS_NH);
        m.vrf = 0; m.nh_family = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) m.nh_addr[k] = 0;
        if (R.vrf) { m.pm_flags |= DP_PM_HAS_VRF; m.vrf = R.vrf & 0x7fffffffu; }
        meta_nh(Img{img_base, *im}, R.nh_ref, m);
        meta[R.idx] = m;
      }
    }
    out[R.idx] = o;
  }
}

// dp_flow_apply: the burst's invalidations (FlowInfo::invalidate_pair,
// net/src/flows/flow_info.rs:435-455) become the flows' status; the marks
// return to idle.
__global__ void __launch_bounds__(256) dp_flow_apply(dpf::FlowCtx fc) {
  const uint32_t cnt = fc.events[0];
  for (uint32_t r = blockIdx.x * 256 + threadIdx.x; r < cnt; r += gridDim.x * 256) {
    const uint32_t c = fc.events[1 + 2 * r], tag = fc.events[2 + 2 * r];
    dpf::FlowSlot &s = fc.slots[c];
    // the fill the event is about (a slot is never refilled while a burst
    // runs -- dp_flow_table's order -- but an event must not be able to
    // cancel an unrelated later flow)
    if (s.state != tag) continue;
    s.status = DP_FLOW_CANCELLED;
    s.mark = dpf::kIdleMark;
    const uint32_t rel = s.related;
    if (rel <= fc.mask && fc.slots[rel].state == s.related_tag) fc.slots[rel].status = DP_FLOW_CANCELLED;
  }
}

// Sum (and clear) the partial histograms into the caller's DoneReason
// counts: block r sums reason r's DPD_STAT_SLOTS partials.
__global__ void __launch_bounds__(DPD_STAT_SLOTS) dp_stats_reduce(unsigned long long *__restrict__ part,
                                                                  unsigned long long *__restrict__ stats) {
  __shared__ unsigned long long wsum[DPD_STAT_SLOTS / 64];
  const int r = blockIdx.x, k = threadIdx.x;
  unsigned long long v = part[r * DPD_STAT_SLOTS + k];
  if (v) part[r * DPD_STAT_SLOTS + k] = 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((k & 63) == 0) wsum[k >> 6] = v;
  __syncthreads();
  if (k == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < DPD_STAT_SLOTS / 64; w++) t += wsum[w];
    if (t) atomicAdd(&stats[r], t);
  }
}
#endif  // DP_IN_PART(0)
#endif

}  // namespace

#ifdef DP_EMU
#ifdef DP_TRIPS
static uint16_t *dp_trip_out;  // per packet x 8 stages (dpemu_trips_out)
#endif
// Host emulation entry (tests/emu only): runs the per-packet body serially.
extern "C" void dpemu_run(const uint8_t *img_base, const void *image_struct, uint8_t *buf,
                          uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta,
                          uint32_t n) {
  thread_local uint8_t slab[SLAB + 16];
  thread_local uint8_t hs[64];
  Img g{img_base, *reinterpret_cast<const Image *>(image_struct)};
  for (uint32_t i = 0; i < n; i++) {
#ifdef DP_TRIPS
    for (int k = 0; k < 8; k++) dp_trip[k] = 0;
    dp_trip_st = 0;
#endif
    const int nch = frame_ok(in[i], buf_bytes) ? window_chunks(in[i]) : 0;
    const uint4 *src = reinterpret_cast<const uint4 *>(buf + (in[i].off & ~15u));
    for (int c = 0; c < nch; c++) {
      const uint4 q = src[c];
      uint32_t *d = reinterpret_cast<uint32_t *>(slab + 16 * c);
      d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w;
    }
    int fl0, fl1;
    const bool fit = (in[i].off & 15) + in[i].len <= (uint32_t)WIN && !(in[i].off & 1);
    FlowPk fp;
    dp_pkt_meta_t *pm = meta ? meta + i : nullptr;
    if (pm) {
      if (fit) process_packet<false, true>(g, slab, hs, buf, buf_bytes, in[i], out[i], pm, fl0, fl1, true, nullptr, fp, i);
      else process_packet<false, true>(g, slab, hs, buf, buf_bytes, in[i], out[i], pm, fl0, fl1, false, nullptr, fp, i);
    } else {
      if (fit) process_packet<false, false>(g, slab, hs, buf, buf_bytes, in[i], out[i], pm, fl0, fl1, true, nullptr, fp, i);
      else process_packet<false, false>(g, slab, hs, buf, buf_bytes, in[i], out[i], pm, fl0, fl1, false, nullptr, fp, i);
    }
    if (fl1 > fl0) flush_range(buf + (in[i].off & ~15u), slab, fl0, fl1);
#ifdef DP_TRIPS
    if (dp_trip_out)
      for (int k = 0; k < 8; k++) dp_trip_out[8 * (uint64_t)i + k] = dp_trip[k];
#endif
  }
}
#ifdef DP_TRIPS
extern "C" void dpemu_trips_out(uint16_t *p) { dp_trip_out = p; }
#endif
#else
// Launch wrappers used by the runtime (dp_runtime.cpp).  The pipeline
// kernel's six instantiations (flows FL, meta MT, replay RP) each have a
// runner; the split build compiles each in its own translation unit.
#define DP_RUN_ARGS                                                                                             \
  uint32_t blocks, hipStream_t s, const uint8_t *img_base, const Image *im, uint8_t *buf, uint64_t buf_bytes, \
      const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n, unsigned long long *part,   \
      const dpf::FlowCtx &fc
// (the kernel's last template argument names the unit's build: DP_V6W, + 2
// without stateful NAT, + 4 with the context tables in LDS; each unit sizes
// its own grid by its TPB, the `blocks` argument is unused)
// The grid of a pipeline launch: one workgroup per TPB packets, or (DP_PERSIST,
// the non-flow kernel) as many as the chip keeps resident -- each then takes
// chunk after chunk, its context-table copy loaded once
static inline uint32_t pipeline_grid(uint32_t chunks, bool fl) {
  if (!DP_PERSIST || fl) return chunks;
  static int cus = 0;
  if (!cus) {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    cus = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  const uint32_t k = (uint32_t)cus * (768u / TPB);  // 3 waves / SIMD: 12 waves per CU
  return chunks < k ? chunks : k;
}
#define DP_RUNNER(NAME, FL, MT, RP)                                                                   \
  extern "C" void NAME(DP_RUN_ARGS) {                                                                 \
    hipLaunchKernelGGL((dp_pipeline_kernel<FL, MT, RP, DP_V6W + (DP_SNAT ? 0 : 2) + (DP_CTX ? 4 : 0)>),      \
                       dim3(pipeline_grid((n + TPB - 1) / TPB, FL)), dim3(TPB), 0, s, img_base, im,  \
                       buf, buf_bytes, in, out, meta, n, part, fc);                                   \
  }
extern "C" {
void dpk_run_pipeline_000(DP_RUN_ARGS);
void dpk_run_pipeline_010(DP_RUN_ARGS);
void dpk_run_pipeline_000w(DP_RUN_ARGS);
void dpk_run_pipeline_010w(DP_RUN_ARGS);
void dpk_run_pipeline_100(DP_RUN_ARGS);
void dpk_run_pipeline_110(DP_RUN_ARGS);
void dpk_run_pipeline_101(DP_RUN_ARGS);
void dpk_run_pipeline_111(DP_RUN_ARGS);
void dpk_run_pipeline_100s(DP_RUN_ARGS);
void dpk_run_pipeline_110s(DP_RUN_ARGS);
void dpk_run_pipeline_100c(DP_RUN_ARGS);
void dpk_run_pipeline_110c(DP_RUN_ARGS);
void dpk_run_pipeline_000n(DP_RUN_ARGS);
void dpk_run_pipeline_010n(DP_RUN_ARGS);
void dpk_run_pipeline_000wn(DP_RUN_ARGS);
void dpk_run_pipeline_010wn(DP_RUN_ARGS);
}
#if DP_IN_PART(1)
DP_RUNNER(dpk_run_pipeline_000, false, false, false)
#endif
#if DP_IN_PART(2)
DP_RUNNER(dpk_run_pipeline_010, false, true, false)
#endif
#if DP_IN_PART(7)
DP_RUNNER(dpk_run_pipeline_000w, false, false, false)
#endif
#if DP_IN_PART(8)
DP_RUNNER(dpk_run_pipeline_010w, false, true, false)
#endif
#if DP_IN_PART(3)
DP_RUNNER(dpk_run_pipeline_100, true, false, false)
#endif
#if DP_IN_PART(4)
DP_RUNNER(dpk_run_pipeline_110, true, true, false)
#endif
#if DP_IN_PART(5)
DP_RUNNER(dpk_run_pipeline_101, true, false, true)
#endif
#if DP_IN_PART(6)
DP_RUNNER(dpk_run_pipeline_111, true, true, true)
#endif
#if DP_PART == 11 || DP_PART < 0  // (a one-unit build: the one instantiation under every name)
DP_RUNNER(dpk_run_pipeline_000n, false, false, false)
#endif
#if DP_PART == 12 || DP_PART < 0
DP_RUNNER(dpk_run_pipeline_010n, false, true, false)
#endif
#if DP_PART == 13 || DP_PART < 0
DP_RUNNER(dpk_run_pipeline_000wn, false, false, false)
#endif
#if DP_PART == 14 || DP_PART < 0
DP_RUNNER(dpk_run_pipeline_010wn, false, true, false)
#endif
#if DP_PART == 9 || DP_PART < 0  // (a one-unit build: the full variant under the lean name)
DP_RUNNER(dpk_run_pipeline_100s, true, false, false)
#endif
#if DP_PART == 10 || DP_PART < 0
DP_RUNNER(dpk_run_pipeline_110s, true, true, false)
#endif
#if DP_PART == 15 || DP_PART < 0  // (the full flows first pass with the context tables in LDS)
DP_RUNNER(dpk_run_pipeline_100c, true, false, false)
#endif
#if DP_PART == 16 || DP_PART < 0
DP_RUNNER(dpk_run_pipeline_110c, true, true, false)
#endif
#if DP_IN_PART(0)
#if defined(DP_TIMING)
extern "C" int dp_debug_stage_cycles(unsigned long long *out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stage_cycles), 16 * sizeof(unsigned long long)) != hipSuccess) return -5;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stage_cycles), z, sizeof(z)) != hipSuccess) return -5;
  }
  return 0;
}
#endif
// Whole-burst failure: every packet InternalFailure (dpgpu.h conventions).
__global__ void __launch_bounds__(256) dp_mark_failed(const dp_pkt_in_t *__restrict__ in,
                                                      dp_pkt_out_t *__restrict__ out,
                                                      dp_pkt_meta_t *__restrict__ meta, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  out[i] = out_record(in[i].off, in[i].len, DP_DONE_INTERNAL_FAILURE);
  if (meta) meta[i] = meta_none();
}

// Compact host staging (dp_process_burst, staged copies).  Packet i's span
// is [in.off & ~15, (in.off + in.len + 15) & ~15) of the burst buffer; the
// host sends the spans back to back (span i at 16 * pos[i] of `cin`).
// dp_stage_expand puts each span at its own offset of the device burst
// buffer; dp_stage_collect packs [span start - grow, span end) of every
// packet at 16 * pos[i] + grow * i of `cout` (grow: DP_HEADROOM when an output may
// start in front of its frame -- VXLAN encap -- else 0).  One wave per 64
// packets, each lane its own packet's 16-byte chunks.
__device__ __forceinline__ uint32_t span_lo(const dp_pkt_in_t &p) { return p.off & ~15u; }
__device__ __forceinline__ uint32_t span_hi(const dp_pkt_in_t &p) { return (p.off + p.len + 15u) & ~15u; }

__global__ void __launch_bounds__(256) dp_stage_expand(const uint8_t *__restrict__ cin, const uint32_t *__restrict__ pos,
                                                       const dp_pkt_in_t *__restrict__ in, uint8_t *__restrict__ buf,
                                                       uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const dp_pkt_in_t p = in[i];
  const uint4 *s = reinterpret_cast<const uint4 *>(cin + 16ull * pos[i]);
  uint4 *d = reinterpret_cast<uint4 *>(buf + span_lo(p));
  const uint32_t c = (span_hi(p) - span_lo(p)) >> 4;
  for (uint32_t k = 0; k < c; k++) d[k] = s[k];
}

__global__ void __launch_bounds__(256) dp_stage_collect(const uint8_t *__restrict__ buf, const uint32_t *__restrict__ pos,
                                                        const dp_pkt_in_t *__restrict__ in, uint8_t *__restrict__ cout,
                                                        uint32_t grow, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const dp_pkt_in_t p = in[i];
  const uint4 *s = reinterpret_cast<const uint4 *>(buf + span_lo(p) - grow);
  uint4 *d = reinterpret_cast<uint4 *>(cout + 16ull * pos[i] + (uint64_t)grow * i);
  const uint32_t c = (span_hi(p) - span_lo(p) + grow) >> 4;
  for (uint32_t k = 0; k < c; k++) d[k] = s[k];
}

extern "C" int dpk_stage_expand(const uint8_t *cin, const uint32_t *pos, const dp_pkt_in_t *in, uint8_t *buf,
                                uint32_t n, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(dp_stage_expand, dim3((n + 255) / 256), dim3(256), 0, stream, cin, pos, in, buf, n);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int dpk_stage_collect(const uint8_t *buf, const uint32_t *pos, const dp_pkt_in_t *in, uint8_t *cout,
                                 uint32_t grow, uint32_t n, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(dp_stage_collect, dim3((n + 255) / 256), dim3(256), 0, stream, buf, pos, in, cout, grow, n);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int dpk_acl_classify(const uint8_t *img_base, const void *image_dev, const dp_acl_key_t *keys,
                                dp_acl_result_t *out, uint32_t n, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(dp_acl_classify_k, dim3((n + 255) / 256), dim3(256), 0, stream, img_base,
                     reinterpret_cast<const Image *>(image_dev), keys, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int dpk_ff_classify(const uint8_t *img_base, const void *image_dev, const dp_ff_input_t *in,
                               dp_ff_result_t *out, uint32_t n, int stage, hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(dp_ff_classify_k, dim3((n + 255) / 256), dim3(256), 0, stream, img_base,
                     reinterpret_cast<const Image *>(image_dev), in, out, n, stage);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int dpk_mark_failed(const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n,
                               hipStream_t stream) {
  if (n == 0 || !in || !out) return 0;
  hipLaunchKernelGGL(dp_mark_failed, dim3((n + 255) / 256), dim3(256), 0, stream, in, out, meta, n);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int dpk_launch_pipeline(const uint8_t *img_base, const void *image_dev, uint8_t *buf,
                                   uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                                   dp_pkt_meta_t *meta, uint32_t n, uint64_t *stats, uint64_t *stats_part,
                                   int v6w, int ctx, hipStream_t stream) {
  if (n == 0) return 0;
  const Image *im = reinterpret_cast<const Image *>(image_dev);
  uint32_t blocks = (n + TPB - 1) / TPB;
  unsigned long long *part = stats ? reinterpret_cast<unsigned long long *>(stats_part) : nullptr;
  const dpf::FlowCtx nofc{};
  // an image with v6 windows needs the units that look them up; the others
  // read the context tables from LDS when they fit (ctx != 0)
  if (meta) (v6w ? (ctx ? dpk_run_pipeline_010w : dpk_run_pipeline_010wn)
                 : (ctx ? dpk_run_pipeline_010 : dpk_run_pipeline_010n))(
      blocks, stream, img_base, im, buf, buf_bytes, in, out, meta, n, part, nofc);
  else (v6w ? (ctx ? dpk_run_pipeline_000w : dpk_run_pipeline_000wn)
            : (ctx ? dpk_run_pipeline_000 : dpk_run_pipeline_000n))(
      blocks, stream, img_base, im, buf, buf_bytes, in, out, meta, n, part, nofc);
  if (stats)
    hipLaunchKernelGGL(dp_stats_reduce, dim3(DP_DONE_COUNT), dim3(DPD_STAT_SLOTS), 0, stream, part,
                       reinterpret_cast<unsigned long long *>(stats));
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The flows variant: counters cleared, the pipeline, the histogram, then the
// flow fix-up and the invalidations, in stream order.  `fc` points at host
// memory holding the launch's FlowCtx (device pointers inside).
extern "C" int dpk_launch_pipeline_flows(const uint8_t *img_base, const void *image_dev, uint8_t *buf,
                                         uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                                         dp_pkt_meta_t *meta, uint32_t n, uint64_t *stats, uint64_t *stats_part,
                                         const void *fc_host, hipStream_t stream, hipStream_t side,
                                         hipEvent_t fork, hipEvent_t fork2, hipEvent_t join, int fork_at) {
  if (n == 0) return 0;
  dpf::FlowCtx fc = *reinterpret_cast<const dpf::FlowCtx *>(fc_host);
  if (hipMemsetAsync(fc.events, 0, sizeof(uint32_t), stream) != hipSuccess) return -5;
  if (hipMemsetAsync(fc.sens, 0, sizeof(uint32_t), stream) != hipSuccess) return -5;
  if (hipMemsetAsync(fc.pf_cnt, 0, sizeof(uint32_t) * DPF_CNT_WORDS, stream) != hipSuccess) return -5;
  const Image *im = reinterpret_cast<const Image *>(image_dev);
  uint32_t blocks = (n + TPB - 1) / TPB;
  unsigned long long *part = stats ? reinterpret_cast<unsigned long long *>(stats_part) : nullptr;
  fc.replay = 0;
  if (fc.lean) {
    // no stateful NAT (Image.snat clear, no flow of the table ever had NAT
    // state) and no v6 windows: the one pass without that code, and no NAT
    // pass (no packet can reach PortForwarder or Masquerade)
    if (meta) dpk_run_pipeline_110s(blocks, stream, img_base, im, buf, buf_bytes, in, out, meta, n, part, fc);
    else dpk_run_pipeline_100s(blocks, stream, img_base, im, buf, buf_bytes, in, out, meta, n, part, fc);
  } else {
  // first pass (the context tables from LDS when they fit); PortForwarder's
  // records in packet order; the replay of the packets that reached it
  // (dp_nat_resolve's decisions)
  if (meta) (fc.ctx ? dpk_run_pipeline_110c : dpk_run_pipeline_110)(blocks, stream, img_base, im, buf, buf_bytes, in,
                                                                    out, meta, n, part, fc);
  else (fc.ctx ? dpk_run_pipeline_100c : dpk_run_pipeline_100)(blocks, stream, img_base, im, buf, buf_bytes, in, out,
                                                               meta, n, part, fc);
  // the NAT pass: records filed by connection, then resolved
  // (grids of about one chip's worth of resident lanes: a burst with no
  // records leaves at once -- 8192 empty workgroups cost 76 us; more lanes
  // than that did not make the 500k-record burst faster)
  const uint32_t pb = (n + 1023) / 1024 < 256 ? (n + 1023) / 1024 : 256;
  const uint32_t rb0 = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  // the records' packets in packet order (dp_bits_*), then the records
  const uint32_t regions = (n + 1023) / 1024;
  const uint32_t cb = (regions + 255) / 256 < 1024 ? (regions + 255) / 256 : 1024;
  const uint32_t eb = (regions + 3) / 4 < 4096 ? (regions + 3) / 4 : 4096;
  auto order = [&](int which) {
    hipLaunchKernelGGL(dp_bits_count, dim3(cb), dim3(256), 0, stream, fc, which);
    hipLaunchKernelGGL(dp_bits_scan, dim3(1), dim3(1024), 0, stream, fc, which);
    hipLaunchKernelGGL(dp_bits_emit, dim3(eb), dim3(256), 0, stream, fc, which);
    hipLaunchKernelGGL(dp_bits_clear, dim3(cb), dim3(256), 0, stream, fc, which);
  };
  order(0);
  hipLaunchKernelGGL(dp_nat_mark, dim3(rb0), dim3(256), 0, stream, img_base, im, fc);
  hipLaunchKernelGGL(dp_nat_prep, dim3(pb), dim3(1024), 0, stream, img_base, im, fc);
  const uint32_t rb = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  // a mixed burst: may the allocating lane meet a port-forwarding creation's key
  hipLaunchKernelGGL(dp_nat_cross, dim3(rb), dim3(256), 0, stream, fc);
  // (fork_at 3) the steady refreshes dp_nat_prep resolved replay on the side
  // stream now, beside the rest of the NAT pass (fc.replay 4)
  auto replay = [&](hipStream_t s, uint32_t which) {
    fc.replay = which;
    if (meta) dpk_run_pipeline_111(blocks, s, img_base, im, buf, buf_bytes, in, out, meta, n, part, fc);
    else dpk_run_pipeline_101(blocks, s, img_base, im, buf, buf_bytes, in, out, meta, n, part, fc);
  };
  const bool forked = side && fork && fork2 && join && fork_at >= 1 && fork_at <= 3;
  if (forked && fork_at == 3) {
    if (hipEventRecord(fork, stream) != hipSuccess || hipStreamWaitEvent(side, fork, 0) != hipSuccess) return -5;
    replay(side, 4);
  }
  // port forwarding near the capacity: the creations' admissions in packet order
  hipLaunchKernelGGL(dp_nat_admit_plan, dim3(rb), dim3(256), 0, stream, img_base, im, fc);
  const uint32_t ab = (n + kAdmChunk - 1) / kAdmChunk;
  hipLaunchKernelGGL(dp_nat_admit_scan, dim3(ab), dim3(1024), 0, stream, fc, 0);
  hipLaunchKernelGGL(dp_nat_admit_scan, dim3(1), dim3(1024), 0, stream, fc, 1);
  hipLaunchKernelGGL(dp_nat_admit_scan, dim3(ab), dim3(1024), 0, stream, fc, 2);
  hipLaunchKernelGGL(dp_nat_resolve<true>, dim3(1), dim3(64), 0, stream, img_base, im, fc);
  hipLaunchKernelGGL(dp_nat_resolve<false>, dim3(rb), dim3(256), 0, stream, img_base, im, fc);
  // The replay of the records off the allocating lane (every record but a
  // masquerade split's lane records: dp_nat_resolve decided them) on the side
  // stream, beside the lane -- forked after the resolve (fork_at 1) or after
  // the lane's plan (2); then the lane's records after it.  Without a side
  // stream, one replay of every record after the lane.
  auto fork_off = [&]() {
    if (hipEventRecord(fork2, stream) != hipSuccess || hipStreamWaitEvent(side, fork2, 0) != hipSuccess) return false;
    replay(side, fork_at == 3 ? 5 : 2);
    return hipEventRecord(join, side) == hipSuccess;
  };
  if (forked && fork_at == 1 && !fork_off()) return -5;
  // a masquerading burst's allocating lane (its records in packet order)
  order(1);
  hipLaunchKernelGGL(dp_nat_lane_plan, dim3(rb), dim3(256), 0, stream, img_base, im, fc);
  if (forked && fork_at >= 2 && !fork_off()) return -5;
  hipLaunchKernelGGL(dp_nat_lane, dim3(1), dim3(64), 0, stream, img_base, im, fc);
  hipLaunchKernelGGL(dp_nat_lane_assign, dim3(rb), dim3(256), 0, stream, fc);
  hipLaunchKernelGGL(dp_nat_pairs, dim3(rb), dim3(256), 0, stream, img_base, im, fc);
  hipLaunchKernelGGL(dp_nat_lane_end, dim3(1), dim3(1), 0, stream, fc);
  if (forked) {
    if (hipStreamWaitEvent(stream, join, 0) != hipSuccess) return -5;
    replay(stream, 3);
  } else {
    replay(stream, 1);
  }
  }
  if (stats)
    hipLaunchKernelGGL(dp_stats_reduce, dim3(DP_DONE_COUNT), dim3(DPD_STAT_SLOTS), 0, stream, part,
                       reinterpret_cast<unsigned long long *>(stats));
  const uint32_t fb = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(dp_flow_fixup, dim3(fb), dim3(256), 0, stream, img_base, im, fc, in, out, meta,
                     reinterpret_cast<unsigned long long *>(stats));
  hipLaunchKernelGGL(dp_flow_apply, dim3(fb), dim3(256), 0, stream, fc);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
#endif  // DP_IN_PART(0)
#endif

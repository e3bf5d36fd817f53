# Development transformation (kept for the record): VXLAN outer headers
# deparsed into LDS at encap; wave-cooperative header-window staging and
# write-back; DoneReason histogram by wave ballots into partial slots.
p = 'dataplane_amd/csrc/dp_kernel.hip'
s = open(p).read()

def rep(old, new):
    global s
    assert s.count(old) == 1, (old[:80], s.count(old))
    s = s.replace(old, new)

def cut(a_mark, b_mark, new, include_b=False):
    global s
    a = s.index(a_mark)
    b = s.index(b_mark, a)
    if include_b:
        b += len(b_mark)
    s = s[:a] + new + s[b:]

rep('''  uint8_t o_fam;
  Addr16 o_src, o_dst;
  uint32_t o_vni;
  uint16_t o_sport, o_len;
  uint8_t o_tos;         // dscp<<2|ecn for the outer header
''', '''  uint8_t o_fam;         // outer IP family; the outer IP/UDP/VXLAN headers are
                         // deparsed at encap into the lane's LDS scratch (F.hs)
''')
rep('''  if (S.encap) { fam = S.o_fam; a = S.o_dst; return; }''', '''  if (S.encap) {  // the outer destination, from the deparsed outer IP header
    fam = S.o_fam;
    const int o = S.o_fam == 4 ? 16 : 24;
    for (int i = 0; i < 4; i++)
      a.w[i] = (S.o_fam == 6 || i == 0)
                   ? ((uint32_t)F.hs[o + 4 * i] << 24) | ((uint32_t)F.hs[o + 4 * i + 1] << 16) |
                         ((uint32_t)F.hs[o + 4 * i + 2] << 8) | F.hs[o + 4 * i + 3]
                   : 0u;
    return;
  }''')
rep('''struct Addr16 { uint32_t w[4]; };  // network order bytes packed big-endian per word
''', '''struct Addr16 { uint32_t w[4]; };  // network order bytes packed big-endian per word

// VXLAN outer header values (IpForwarder::build_vxlan_headers)
struct OuterHdr {
  uint8_t fam, tos;      // outer IP family; dscp<<2|ecn
  uint16_t sport, len;   // UDP source port; UDP length
  uint32_t vni;
  Addr16 src, dst;
};
// 16-bit words of Eth + outer IP + UDP + VXLAN
__device__ __forceinline__ int outer_words(int fam) { return fam == 4 ? 25 : 35; }
__device__ __forceinline__ uint32_t outer_word(const OuterHdr &S, int i, uint32_t ck4);
__device__ __forceinline__ uint32_t outer_ck4(const OuterHdr &S);
''')
rep('''  for (int i = 0; i < 4; i++) {
    S.o_src.w[i] = ((uint32_t)fb.vtep_ip[4 * i] << 24) | ((uint32_t)fb.vtep_ip[4 * i + 1] << 16) | ((uint32_t)fb.vtep_ip[4 * i + 2] << 8) | fb.vtep_ip[4 * i + 3];
    S.o_dst.w[i] = ((uint32_t)in.addr[4 * i] << 24) | ((uint32_t)in.addr[4 * i + 1] << 16) | ((uint32_t)in.addr[4 * i + 2] << 8) | in.addr[4 * i + 3];
  }
  if (S.o_fam == 4) { S.o_src.w[1] = S.o_src.w[2] = S.o_src.w[3] = 0; S.o_dst.w[1] = S.o_dst.w[2] = S.o_dst.w[3] = 0; }''', '''  OuterHdr ob;
  for (int i = 0; i < 4; i++) {
    ob.src.w[i] = ((uint32_t)fb.vtep_ip[4 * i] << 24) | ((uint32_t)fb.vtep_ip[4 * i + 1] << 16) | ((uint32_t)fb.vtep_ip[4 * i + 2] << 8) | fb.vtep_ip[4 * i + 3];
    ob.dst.w[i] = ((uint32_t)in.addr[4 * i] << 24) | ((uint32_t)in.addr[4 * i + 1] << 16) | ((uint32_t)in.addr[4 * i + 2] << 8) | in.addr[4 * i + 3];
  }
  if (S.o_fam == 4) { ob.src.w[1] = ob.src.w[2] = ob.src.w[3] = 0; ob.dst.w[1] = ob.dst.w[2] = ob.dst.w[3] = 0; }''')
rep('''  S.o_sport = (uint16_t)(x % 16384 + 49152);
  S.o_len = (uint16_t)((F.len - S.pay_start) + H.size + 16);
  S.o_tos = S.has_dscp ? (uint8_t)((S.dscp << 2) | S.ecn) : 0;
  S.o_vni = in.vni;
''', '''  ob.sport = (uint16_t)(x % 16384 + 49152);
  ob.len = (uint16_t)((F.len - S.pay_start) + H.size + 16);
  ob.tos = S.has_dscp ? (uint8_t)((S.dscp << 2) | S.ecn) : 0;
  ob.vni = in.vni;
  ob.fam = S.o_fam;
  // deparse the outer IP/UDP/VXLAN now, over the dead hash input: none of it
  // stays live in registers until serialize (Egress adds the outer Ethernet)
  const int nw = outer_words(ob.fam);
  const uint32_t ck4 = outer_ck4(ob);
#pragma unroll 1
  for (int i = 7; i < nw; i++) {
    const uint32_t v = outer_word(ob, i, ck4);
    F.hs[2 * (i - 7)] = (uint8_t)(v >> 8);
    F.hs[2 * (i - 7) + 1] = (uint8_t)v;
  }
''')
cut('// 16-bit word i of the VXLAN outer headers (Eth + IPv4/IPv6 + UDP + VXLAN)', '// --- serializer', r'''// 16-bit word i >= 7 of the VXLAN outer headers (Eth + IPv4/IPv6 + UDP +
// VXLAN; words 0-6, the outer Ethernet, come from Egress)
__device__ __forceinline__ uint32_t outer_word(const OuterHdr &S, int i, uint32_t ck4) {
  int j = i - 7;
  if (S.fam == 4) {
    if (j < 10) {
      switch (j) {
        case 0: return 0x4500u | S.tos;
        case 1: return (20u + S.len) & 0xffff;
        case 2: return 0;
        case 3: return 0x4000u;              // Ipv4Header::default(): DF
        case 4: return (64u << 8) | 17u;
        case 5: return ck4;
        case 6: return S.src.w[0] >> 16;
        case 7: return S.src.w[0] & 0xffff;
        case 8: return S.dst.w[0] >> 16;
        default: return S.dst.w[0] & 0xffff;
      }
    }
    j -= 10;
  } else {
    if (j < 20) {
      if (j == 0) return ((0x60u | (S.tos >> 4)) << 8) | ((S.tos & 0xfu) << 4);
      if (j == 1) return 0;
      if (j == 2) return S.len;
      if (j == 3) return (17u << 8) | 64u;
      int k = j - 4;
      uint32_t w = k < 8 ? aw(S.src, k >> 1) : aw(S.dst, (k - 8) >> 1);
      return (k & 1) ? (w & 0xffff) : (w >> 16);
    }
    j -= 20;
  }
  switch (j) {
    case 0: return S.sport;
    case 1: return 4789u;
    case 2: return S.len;
    case 3: return 0;                        // outer UDP checksum 0
    case 4: return 0x0800u;                  // VXLAN flags: I
    case 5: return 0;
    case 6: return (S.vni >> 8) & 0xffff;
    default: return (S.vni & 0xff) << 8;
  }
}

// outer IPv4 header checksum (0 for an IPv6 outer header)
__device__ __forceinline__ uint32_t outer_ck4(const OuterHdr &S) {
  if (S.fam != 4) return 0;
  uint64_t t = 0x4500u | S.tos;
  t += (uint16_t)(20 + S.len); t += 0x4000; t += (64u << 8) | 17;
  t += (S.src.w[0] >> 16) + (S.src.w[0] & 0xffff) + (S.dst.w[0] >> 16) + (S.dst.w[0] & 0xffff);
  return (uint16_t)~fold(t);
}

''')
cut('// Write window bytes [a, e) (frame-relative) back to the burst buffer,', '// Packet::serialize (net/src/packet/mod.rs:342-374)', r'''// Window positions [p, we) of one slab back to the burst buffer (gbase: the
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

''')
rep('''__device__ __forceinline__ int serialize(const Frame &F, const Hdr &H0, State &S) {
''', '''__device__ __forceinline__ int serialize(const Frame &F, const Hdr &H0, State &S, int &fl0, int &fl1) {
  fl0 = fl1 = 0;
''')
cut('''  if (S.encap) {
    const int nw = S.o_fam == 4 ? 25 : 35;''', '''  flush_window(F, start, H.hb + H.size);
  return start;
}''', r'''  if (S.encap) {  // outer Ethernet (Egress), then the outer IP/UDP/VXLAN deparsed at encap
    wput_mac(F, start, S.odst);
    wput_mac(F, start + 6, S.osrc);
    wput16(F, start + 12, S.o_fam == 4 ? 0x0800u : 0x86ddu);
    const int nb = 2 * (outer_words(S.o_fam) - 7);
#pragma unroll 1
    for (int i = 0; i < nb; i++) wput8(F, start + 14 + i, F.hs[i]);
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
}''', include_b=True)
rep('''const dp_pkt_in_t &pin, dp_pkt_out_t &o) {''', '''const dp_pkt_in_t &pin, dp_pkt_out_t &o, int &fl0, int &fl1) {
  fl0 = fl1 = 0;''')
rep('''  if (pin.off < DP_HEADROOM || (((uint64_t)pin.off + pin.len + 15) & ~15ull) > buf_bytes) {''',
    '''  if (!frame_ok(pin, buf_bytes)) {''')
cut('  // stage the header window: 16-byte loads, stored as 4 dword LDS writes', '  o.off = pin.off; o.len = pin.len; o.acl = 0;',
    '  // the header window is staged in `slab` by the caller (kernel / dpemu_run)\n')
rep('      int st = serialize(F, H, S);', '      int st = serialize(F, H, S, fl0, fl1);')
cut('// occupancy target: the compiler keeps VGPRs within 512 / DP_WAVES', '#endif\n\n}  // namespace', r'''// occupancy target: the compiler keeps VGPRs within 512 / DP_WAVES
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
      const uint4 v = *reinterpret_cast<const uint4 *>(buf + qb + 16 * c);
      lds_u32 *d = (lds_u32 *)(slab_wave + q * SLAB + 16 * c);
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  }
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
      *reinterpret_cast<uint4 *>(buf + qb + 16 * c) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

__global__ void __launch_bounds__(TPB) DP_OCC
dp_pipeline_kernel(const uint8_t *__restrict__ img_base, Image im, uint8_t *__restrict__ buf,
                   uint64_t buf_bytes, const dp_pkt_in_t *__restrict__ in,
                   dp_pkt_out_t *__restrict__ out, uint32_t n, unsigned long long *__restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_all[TPB * (SLAB + HS)];
  uint8_t *slab_all = lds_all;
  uint8_t *hash_all = lds_all + TPB * SLAB;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  uint8_t *slab_wave = slab_all + (tid - lane) * SLAB;
  lds_u8 *slab = (lds_u8 *)(slab_all + tid * SLAB);
  const uint32_t i = blockIdx.x * TPB + tid;
  const bool live = i < n;
  dp_pkt_in_t pin{};
  if (live) pin = in[i];
  const uint32_t base = pin.off & ~15u;
  const int nch = live && frame_ok(pin, buf_bytes) ? window_chunks(pin) : 0;
  wave_load_windows(buf, slab_wave, base, nch);
  __syncthreads();
  uint8_t done_code = DONE_NONE;
  int fl0 = 0, fl1 = 0;
  if (live) {
    Img g{img_base, im};
    dp_pkt_out_t o;
    done_code = process_packet(g, slab, (lds_u8 *)(hash_all + tid * HS), buf, buf_bytes, pin, o, fl0, fl1);
    out[i] = o;
  }
  __syncthreads();
  // write-back: whole chunks by the wave, a partial tail by its owner
  wave_store_windows(buf, slab_wave, base, fl0 >> 4, fl1 >> 4);
  if (fl1 & 15) flush_range(buf + base, slab, fl1 & ~15, fl1);
  // DoneReason histogram: per wave by ballot, one atomic per reason present
  // into one of DPD_STAT_SLOTS partial histograms (dp_stats_reduce sums them)
  if (part) {
    unsigned long long pending = __ballot(live && done_code < DP_DONE_COUNT);
    const int slot = (int)((blockIdx.x * (TPB / 64) + (tid >> 6)) & (DPD_STAT_SLOTS - 1));
    while (pending) {
      const int leader = __ffsll(pending) - 1;
      const int r = __shfl((int)done_code, leader);
      const unsigned long long m = __ballot(live && (int)done_code == r) & pending;
      if (lane == leader) atomicAdd(&part[slot * DP_DONE_COUNT + r], (unsigned long long)__popcll(m));
      pending &= ~m;
    }
  }
}

// Sum (and clear) the partial histograms into the caller's DoneReason counts.
__global__ void __launch_bounds__(64) dp_stats_reduce(unsigned long long *__restrict__ part,
                                                      unsigned long long *__restrict__ stats) {
  const int r = threadIdx.x;
  if (r >= DP_DONE_COUNT) return;
  unsigned long long s = 0;
  for (int k = 0; k < DPD_STAT_SLOTS; k++) {
    s += part[k * DP_DONE_COUNT + r];
    part[k * DP_DONE_COUNT + r] = 0;
  }
  if (s) atomicAdd(&stats[r], s);
}
''')
rep('''  for (uint32_t i = 0; i < n; i++) process_packet(g, slab, hs, buf, buf_bytes, in[i], out[i]);''',
    '''  for (uint32_t i = 0; i < n; i++) {
    const int nch = frame_ok(in[i], buf_bytes) ? window_chunks(in[i]) : 0;
    const uint4 *src = reinterpret_cast<const uint4 *>(buf + (in[i].off & ~15u));
    for (int c = 0; c < nch; c++) {
      const uint4 q = src[c];
      uint32_t *d = reinterpret_cast<uint32_t *>(slab + 16 * c);
      d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w;
    }
    int fl0, fl1;
    process_packet(g, slab, hs, buf, buf_bytes, in[i], out[i], fl0, fl1);
    if (fl1 > fl0) flush_range(buf + (in[i].off & ~15u), slab, fl0, fl1);
  }''')
a = s.index('extern "C" int dpk_launch_pipeline(')
s = s[:a] + r'''extern "C" int dpk_launch_pipeline(const uint8_t *img_base, const void *image_struct, uint8_t *buf,
                                   uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                                   uint32_t n, uint64_t *stats, uint64_t *stats_part, hipStream_t stream) {
  if (n == 0) return 0;
  Image im = *reinterpret_cast<const Image *>(image_struct);
  uint32_t blocks = (n + TPB - 1) / TPB;
  unsigned long long *part = stats ? reinterpret_cast<unsigned long long *>(stats_part) : nullptr;
  hipLaunchKernelGGL(dp_pipeline_kernel, dim3(blocks), dim3(TPB), 0, stream, img_base, im, buf,
                     buf_bytes, in, out, n, part);
  if (stats)
    hipLaunchKernelGGL(dp_stats_reduce, dim3(1), dim3(64), 0, stream, part,
                       reinterpret_cast<unsigned long long *>(stats));
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
#endif
'''
open(p, 'w').write(s)

d = 'dataplane_amd/csrc/dp_device.h'
t = open(d).read()
assert '#define DPD_MAX_INSTR 4' in t
t = t.replace('#define DPD_MAX_INSTR 4', '#define DPD_MAX_INSTR 4\n// partial DoneReason histograms per context (kernel atomics spread over slots)\n#define DPD_STAT_SLOTS 256', 1)
open(d, 'w').write(t)

r = 'dataplane_amd/csrc/dp_runtime.cpp'
t = open(r).read()
def rr(old, new):
    global t
    assert t.count(old) == 1, old[:60]
    t = t.replace(old, new)
rr('''                                   uint32_t n, uint64_t *stats, hipStream_t stream);''',
   '''                                   uint32_t n, uint64_t *stats, uint64_t *stats_part, hipStream_t stream);''')
rr('''  uint64_t *d_stats = nullptr;
  uint32_t cap_n = 0;''', '''  uint64_t *d_stats = nullptr;
  uint64_t *d_part = nullptr;        // partial DoneReason histograms (kernel side)
  uint32_t cap_n = 0;''')
rr('''    return fail(DP_ENOMEM, "hipMalloc stats", e);
  *out = c.release();''', '''    return fail(DP_ENOMEM, "hipMalloc stats", e);
  const size_t part_bytes = sizeof(uint64_t) * DP_DONE_COUNT * DPD_STAT_SLOTS;
  if ((e = hipMalloc(&c->d_part, part_bytes)) != hipSuccess) return fail(DP_ENOMEM, "hipMalloc stats partials", e);
  if ((e = hipMemset(c->d_part, 0, part_bytes)) != hipSuccess) return fail(DP_EIO, "clear stats partials", e);
  *out = c.release();''')
rr('''  if (c->d_stats) (void)hipFree(c->d_stats);''', '''  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->d_part) (void)hipFree(c->d_part);''')
rr('''dev_out, n, dev_stats, s);''', '''dev_out, n, dev_stats, c->d_part, s);''')
open(r, 'w').write(t)
print("applied")

// SPDX-License-Identifier: Apache-2.0
//
// DPDK rx / tx burst glue (include/dpgpu.h "DPDK rx / tx burst glue"): the
// translation between an rx burst of rte_mbufs and the path's burst records,
// and back.  The reference reads a frame as buf_addr + data_off, data_len
// bytes of the first segment (Mbuf::raw_data, dpdk/src/mem.rs:502-522) and
// grows / shrinks it in the mbuf's headroom (rte_pktmbuf_prepend / _adj,
// :547-590); the GPU path rewrites frames in place inside their headroom, so
// a delivered mbuf only needs data_off / data_len / pkt_len updated.
#include <cstdint>
#include <cstring>

#include "../../include/dpgpu.h"

namespace {

template <class T> T rd(const void *m, uint16_t off) {
  T v;
  memcpy(&v, static_cast<const uint8_t *>(m) + off, sizeof(T));
  return v;
}
template <class T> void wr(void *m, uint16_t off, T v) {
  memcpy(static_cast<uint8_t *>(m) + off, &v, sizeof(T));
}

// A record frame_ok rejects: the packet ends InternalFailure, untouched.
dp_pkt_in_t bad_record() {
  dp_pkt_in_t r{};
  r.off = 0;
  r.len = 0;
  return r;
}

}  // namespace

extern "C" {

int dp_mbuf_burst_in(const void *pool_base, uint64_t pool_bytes, void *const *mbufs, uint32_t n,
                     const dp_mbuf_layout_t *layout, const uint32_t *port_ifindex, uint32_t n_ports,
                     dp_pkt_in_t *in) {
  if (!pool_base || (!mbufs && n) || !layout || (!in && n)) return DP_EINVAL;
  const uintptr_t base = reinterpret_cast<uintptr_t>(pool_base);
  for (uint32_t i = 0; i < n; i++) {
    const void *m = mbufs[i];
    if (!m) { in[i] = bad_record(); continue; }
    const uintptr_t buf = rd<uintptr_t>(m, layout->buf_addr);
    const uint16_t doff = rd<uint16_t>(m, layout->data_off);
    const uint16_t dlen = rd<uint16_t>(m, layout->data_len);
    const uint16_t port = rd<uint16_t>(m, layout->port);
    const uintptr_t frame = buf + doff;
    // the headroom in front of the frame belongs to the packet (DP_HEADROOM
    // contract): it must lie in the pool region, as must the frame rounded
    // up to 16 bytes (the kernel stages frames with 16-byte loads): a frame
    // at the very end of the pool fails alone, not the whole burst
    if (buf < base || doff < DP_HEADROOM || frame - base > UINT32_MAX ||
        ((frame - base + dlen + 15) & ~(uintptr_t)15) > pool_bytes) {
      in[i] = bad_record();
      continue;
    }
    dp_pkt_in_t r{};
    r.off = static_cast<uint32_t>(frame - base);
    r.len = dlen;
    r.flags = 0;
    r.iif = port_ifindex ? (port < n_ports ? port_ifindex[port] : 0) : port;
    r.src_vni = 0;
    in[i] = r;
  }
  return 0;
}

int dp_mbuf_burst_out(void *const *mbufs, uint32_t n, const dp_mbuf_layout_t *layout, const dp_pkt_in_t *in,
                      const dp_pkt_out_t *out) {
  if ((!mbufs && n) || !layout || (!in && n) || (!out && n)) return DP_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    if (!mbufs[i] || out[i].done != DP_DONE_DELIVERED || in[i].off < DP_HEADROOM) continue;
    void *m = mbufs[i];
    // the serialized frame starts out.off - in.off bytes from the received one
    const int64_t doff = (int64_t)rd<uint16_t>(m, layout->data_off) + ((int64_t)out[i].off - (int64_t)in[i].off);
    if (doff < 0 || doff > UINT16_MAX) return DP_EINVAL;  // cannot happen within the headroom contract
    // rte_pktmbuf_prepend / rte_pktmbuf_adj move data_len and pkt_len together
    const int64_t grow = (int64_t)out[i].len - (int64_t)rd<uint16_t>(m, layout->data_len);
    wr<uint16_t>(m, layout->data_off, static_cast<uint16_t>(doff));
    wr<uint16_t>(m, layout->data_len, out[i].len);
    wr<uint32_t>(m, layout->pkt_len, static_cast<uint32_t>((int64_t)rd<uint32_t>(m, layout->pkt_len) + grow));
  }
  return 0;
}

}  // extern "C"

// TEST INFRASTRUCTURE (see dp_emu_shim.h).
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "../../dataplane_amd/csrc/dp_tables.h"

extern "C" void dpemu_run(const uint8_t *img_base, const void *image_struct, uint8_t *buf,
                          uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta,
                          uint32_t n);

extern "C" int dpemu_process(const dp_tables_desc_t *d, uint8_t *buf, uint64_t buf_bytes,
                             const dp_pkt_in_t *in, dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n) {
  dpd::BuiltImage bi;
  int rc = dpd::build_image(d, bi);
  if (rc) return rc;
  uint64_t padded = ((buf_bytes + 15) & ~15ull) + 16;
  std::vector<uint8_t> store(padded + 16);
  uint8_t *al = reinterpret_cast<uint8_t *>(((uintptr_t)store.data() + 15) & ~(uintptr_t)15);
  memcpy(al, buf, buf_bytes);
  // the image is position independent (offsets); align its host copy too
  std::vector<uint8_t> img(bi.bytes.size() + 16);
  uint8_t *ib = reinterpret_cast<uint8_t *>(((uintptr_t)img.data() + 15) & ~(uintptr_t)15);
  memcpy(ib, bi.bytes.data(), bi.bytes.size());
  dpemu_run(ib, &bi.im, al, padded, in, out, meta, n);
  memcpy(buf, al, buf_bytes);
  return 0;
}

// (n_vni_slots, pair map slots, pair records, next hops, LDS context bytes)
extern "C" int dpemu_image_ctx(const dp_tables_desc_t *d, uint32_t *o) {
  dpd::BuiltImage bi;
  if (dpd::build_image(d, bi)) return -1;
  const dpd::Image &im = bi.im;
  o[0] = im.vni_mask + 1; o[1] = im.pairs.mask + 1; o[2] = im.n_pair_recs; o[3] = im.n_nh; o[4] = im.ctx_bytes;
  return 0;
}
extern "C" uint64_t dpemu_image_bytes(const dp_tables_desc_t *d) {
  dpd::BuiltImage bi;
  if (dpd::build_image(d, bi)) return 0;
  return bi.bytes.size();
}

// CPU leg of bench.py's baseline: the kernel's per-packet body over the same
// compiled table image, on `threads` host threads, bursts of `burst` packets
// taken from a shared counter (as DPDK workers take rx bursts).
struct dpemu_ctx {
  dpd::BuiltImage bi;
  std::vector<uint8_t> img;
  uint8_t *ib = nullptr;
};

extern "C" void *dpemu_ctx_create(const dp_tables_desc_t *d) {
  auto *c = new dpemu_ctx;
  if (dpd::build_image(d, c->bi)) { delete c; return nullptr; }
  c->img.resize(c->bi.bytes.size() + 16);
  c->ib = reinterpret_cast<uint8_t *>(((uintptr_t)c->img.data() + 15) & ~(uintptr_t)15);
  memcpy(c->ib, c->bi.bytes.data(), c->bi.bytes.size());
  return c;
}

extern "C" void dpemu_ctx_free(void *c) { delete static_cast<dpemu_ctx *>(c); }

// `buf` must be 16-byte aligned with 16 bytes of slack past buf_bytes.
extern "C" int dpemu_run_parallel(void *cv, uint8_t *buf, uint64_t buf_bytes, const dp_pkt_in_t *in,
                                  dp_pkt_out_t *out, dp_pkt_meta_t *meta, uint32_t n, uint32_t burst,
                                  uint32_t threads) {
  auto *c = static_cast<dpemu_ctx *>(cv);
  if (!c || !threads || !burst || ((uintptr_t)buf & 15)) return -22;
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < threads; k++)
    th.emplace_back([&]() {
      for (;;) {
        const uint32_t s = next.fetch_add(burst);
        if (s >= n) break;
        const uint32_t e = s + burst < n ? s + burst : n;
        dpemu_run(c->ib, &c->bi.im, buf, buf_bytes, in + s, out + s, meta ? meta + s : nullptr, e - s);
      }
    });
  for (auto &t : th) t.join();
  return 0;
}

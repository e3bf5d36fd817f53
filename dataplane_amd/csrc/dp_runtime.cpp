// SPDX-License-Identifier: Apache-2.0
//
// C-ABI implementation (include/dpgpu.h): contexts, table publication and
// burst submission on HIP streams.
//
// Table publication mirrors the reference's lock-free reader handles
// (left-right for FIB / NAT, ArcSwap Slot for flow-filter / ACL,
// SURVEY.md §1): dp_tables_publish compiles and uploads a new image, then
// swaps one per-device shared pointer under a mutex.  Each burst pins the
// image it launched with (a shared_ptr held by the context until its next
// burst), so the previous image is released only after every context has
// moved on; hipFree synchronises, so no kernel still reads freed memory.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "../../include/dpgpu.h"
#include "dp_tables.h"

extern "C" int dpk_launch_pipeline(const uint8_t *img_base, const void *image_struct, uint8_t *buf,
                                   uint64_t buf_bytes, const dp_pkt_in_t *in, dp_pkt_out_t *out,
                                   uint32_t n, uint64_t *stats, uint64_t *stats_part, hipStream_t stream);

namespace {

thread_local std::string g_err;

int fail(int rc, const char *what, hipError_t e = hipSuccess) {
  g_err = what;
  if (e != hipSuccess) {
    g_err += ": ";
    g_err += hipGetErrorString(e);
  }
  return rc;
}

struct DevImage {
  int device = 0;
  uint8_t *dev = nullptr;
  dpd::Image im{};
  ~DevImage() {
    if (dev) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(device);
      (void)hipFree(dev);
      (void)hipSetDevice(prev);
    }
  }
};

struct DeviceTables {
  std::mutex mu;
  std::shared_ptr<DevImage> cur;
};

std::mutex g_dev_mu;
std::map<int, std::unique_ptr<DeviceTables>> g_dev;

DeviceTables &dev_tables(int device) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto &p = g_dev[device];
  if (!p) p.reset(new DeviceTables());
  return *p;
}

}  // namespace

struct dp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::shared_ptr<DevImage> pinned;  // image used by the last burst
  // host-path staging
  uint8_t *d_buf = nullptr;
  uint64_t d_buf_cap = 0;
  dp_pkt_in_t *d_in = nullptr;
  dp_pkt_out_t *d_out = nullptr;
  uint64_t *d_stats = nullptr;
  uint64_t *d_part = nullptr;        // partial DoneReason histograms (kernel side)
  uint32_t cap_n = 0;
};

extern "C" {

uint32_t dp_abi_version(void) { return DPGPU_ABI_VERSION; }

const char *dp_last_error(void) { return g_err.c_str(); }

int dp_ctx_create(int device_ordinal, dp_ctx_t **out) {
  if (!out) return fail(DP_EINVAL, "null out");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(DP_ENODEV, "no HIP device", e);
  if (device_ordinal < 0 || device_ordinal >= ndev) return fail(DP_ENODEV, "bad device ordinal");
  std::unique_ptr<dp_ctx> c(new dp_ctx());
  c->device = device_ordinal;
  if ((e = hipSetDevice(device_ordinal)) != hipSuccess) return fail(DP_EIO, "hipSetDevice", e);
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail(DP_EIO, "hipStreamCreate", e);
  if ((e = hipMalloc(&c->d_stats, sizeof(uint64_t) * DP_DONE_COUNT)) != hipSuccess)
    return fail(DP_ENOMEM, "hipMalloc stats", e);
  const size_t part_bytes = sizeof(uint64_t) * DP_DONE_COUNT * DPD_STAT_SLOTS;
  if ((e = hipMalloc(&c->d_part, part_bytes)) != hipSuccess) return fail(DP_ENOMEM, "hipMalloc stats partials", e);
  if ((e = hipMemset(c->d_part, 0, part_bytes)) != hipSuccess) return fail(DP_EIO, "clear stats partials", e);
  *out = c.release();
  return 0;
}

int dp_ctx_destroy(dp_ctx_t *c) {
  if (!c) return DP_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  c->pinned.reset();
  if (c->d_buf) (void)hipFree(c->d_buf);
  if (c->d_in) (void)hipFree(c->d_in);
  if (c->d_out) (void)hipFree(c->d_out);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->d_part) (void)hipFree(c->d_part);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int dp_tables_publish(dp_ctx_t *c, const dp_tables_desc_t *tables) {
  if (!c || !tables) return fail(DP_EINVAL, "null argument");
  dpd::BuiltImage bi;
  int rc = dpd::build_image(tables, bi);
  if (rc) return fail(rc, "table compile rejected the descriptors");
  (void)hipSetDevice(c->device);
  auto img = std::make_shared<DevImage>();
  img->device = c->device;
  hipError_t e = hipMalloc(&img->dev, bi.bytes.size());
  if (e != hipSuccess) return fail(DP_ENOMEM, "hipMalloc table image", e);
  if ((e = hipMemcpy(img->dev, bi.bytes.data(), bi.bytes.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(DP_EIO, "upload table image", e);
  img->im = bi.im;
  DeviceTables &dt = dev_tables(c->device);
  std::shared_ptr<DevImage> old;
  {
    std::lock_guard<std::mutex> lk(dt.mu);
    old = dt.cur;
    dt.cur = img;
  }
  // `old` is freed here only if no context still pins it
  return 0;
}

int64_t dp_tables_genid(const dp_ctx_t *c) {
  if (!c) return -1;
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> lk(dt.mu);
  return dt.cur ? dt.cur->im.genid : -1;
}

uint64_t dp_tables_device_bytes(const dp_ctx_t *c) {
  if (!c) return 0;
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> lk(dt.mu);
  return dt.cur ? dt.cur->im.bytes : 0;
}

static std::shared_ptr<DevImage> current(dp_ctx_t *c) {
  DeviceTables &dt = dev_tables(c->device);
  std::lock_guard<std::mutex> lk(dt.mu);
  return dt.cur;
}

int dp_process_burst_device(dp_ctx_t *c, uint8_t *dev_buf, uint64_t buf_bytes,
                            const dp_pkt_in_t *dev_in, dp_pkt_out_t *dev_out, uint32_t n,
                            uint64_t *dev_stats, void *stream) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!dev_buf || !dev_in || !dev_out || ((uintptr_t)dev_buf & 15)) return fail(DP_EINVAL, "bad burst buffers");
  auto img = current(c);
  if (!img) return fail(DP_ENOTABLES, "no tables published");
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  int rc = dpk_launch_pipeline(img->dev, &img->im, dev_buf, buf_bytes, dev_in, dev_out, n, dev_stats, c->d_part, s);
  if (rc) return fail(DP_EIO, "kernel launch failed", hipGetLastError());
  c->pinned = img;
  return 0;
}

int dp_process_burst(dp_ctx_t *c, uint8_t *buf, uint64_t buf_bytes, const dp_pkt_in_t *in,
                     dp_pkt_out_t *out, uint32_t n, uint64_t *stats) {
  if (!c) return fail(DP_EINVAL, "null ctx");
  if (n == 0) return 0;
  if (!buf || !in || !out) return fail(DP_EINVAL, "null burst buffers");
  for (uint32_t i = 0; i < n; i++)
    if (in[i].off < DP_HEADROOM || (uint64_t)in[i].off + in[i].len > buf_bytes)
      return fail(DP_EINVAL, "frame outside the burst buffer / headroom");
  (void)hipSetDevice(c->device);
  hipError_t e;
  uint64_t need = ((buf_bytes + 15) & ~15ull) + 16;
  if (need > c->d_buf_cap) {
    if (c->d_buf) (void)hipFree(c->d_buf);
    c->d_buf = nullptr;
    if ((e = hipMalloc(&c->d_buf, need)) != hipSuccess) { c->d_buf_cap = 0; return fail(DP_ENOMEM, "hipMalloc burst", e); }
    c->d_buf_cap = need;
  }
  if (n > c->cap_n) {
    if (c->d_in) (void)hipFree(c->d_in);
    if (c->d_out) (void)hipFree(c->d_out);
    c->d_in = nullptr; c->d_out = nullptr; c->cap_n = 0;
    if ((e = hipMalloc(&c->d_in, sizeof(dp_pkt_in_t) * n)) != hipSuccess) return fail(DP_ENOMEM, "hipMalloc in", e);
    if ((e = hipMalloc(&c->d_out, sizeof(dp_pkt_out_t) * n)) != hipSuccess) return fail(DP_ENOMEM, "hipMalloc out", e);
    c->cap_n = n;
  }
  hipStream_t s = c->stream;
  if ((e = hipMemcpyAsync(c->d_buf, buf, buf_bytes, hipMemcpyHostToDevice, s)) != hipSuccess) return fail(DP_EIO, "H2D burst", e);
  if ((e = hipMemcpyAsync(c->d_in, in, sizeof(dp_pkt_in_t) * n, hipMemcpyHostToDevice, s)) != hipSuccess) return fail(DP_EIO, "H2D meta", e);
  if (stats && (e = hipMemsetAsync(c->d_stats, 0, sizeof(uint64_t) * DP_DONE_COUNT, s)) != hipSuccess) return fail(DP_EIO, "memset stats", e);
  int rc = dp_process_burst_device(c, c->d_buf, need, c->d_in, c->d_out, n, stats ? c->d_stats : nullptr, s);
  if (rc) return rc;
  if ((e = hipMemcpyAsync(buf, c->d_buf, buf_bytes, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(DP_EIO, "D2H burst", e);
  if ((e = hipMemcpyAsync(out, c->d_out, sizeof(dp_pkt_out_t) * n, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(DP_EIO, "D2H meta", e);
  uint64_t hstats[DP_DONE_COUNT];
  if (stats && (e = hipMemcpyAsync(hstats, c->d_stats, sizeof(hstats), hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(DP_EIO, "D2H stats", e);
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(DP_EIO, "stream sync", e);
  if (stats) for (int k = 0; k < DP_DONE_COUNT; k++) stats[k] += hstats[k];
  return 0;
}

int dp_ctx_synchronize(dp_ctx_t *c) {
  if (!c) return DP_EINVAL;
  hipError_t e = hipStreamSynchronize(c->stream);
  return e == hipSuccess ? 0 : fail(DP_EIO, "stream sync", e);
}

}  // extern "C"

// Microbenchmark (diagnostic, not product): price of the packet kernel's
// frame I/O shapes.  2M 64-byte frames in DPDK mbuf slots (192-byte stride,
// frame 64-byte aligned, as bench.py's --layout dpdk), fresh from HBM.
//   lanes/pkt L: 1 (a lane moves its frame as 4 x 16 B), 2 (2 x 16 B each),
//                4 (one 16-byte chunk each: the round-1 cooperative form)
//   mode: load only, or load + store back (each lane stores what it loaded)
// Also the per-packet records: 16 B in-record loads, 32 B / 16 B / 8 B
// out-record stores.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr uint32_t SLOT = 192, HEAD = 128;

template <int L, bool STORE>
__global__ void __launch_bounds__(256) frame_kernel(uint8_t *__restrict__ buf, uint32_t *__restrict__ sink, uint32_t n) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t p = t / L, part = t % L;
  if (p >= n) return;
  uint4 *f = reinterpret_cast<uint4 *>(buf + (uint64_t)p * SLOT + HEAD);
  constexpr int C = 4 / L;
  uint4 v[C];
#pragma unroll
  for (int c = 0; c < C; c++) v[c] = f[part * C + c];
  uint32_t x = 0;
#pragma unroll
  for (int c = 0; c < C; c++) x ^= v[c].x ^ v[c].w;
  if (STORE) {
#pragma unroll
    for (int c = 0; c < C; c++) { v[c].y ^= 1; f[part * C + c] = v[c]; }
  } else if (x == 0x9e3779b9u) {
    sink[t] = x;
  }
}

template <int B>
__global__ void __launch_bounds__(256) rec_kernel(const uint4 *__restrict__ in, uint8_t *__restrict__ out, uint32_t n) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const uint4 r = in[t];
  if (B == 0) return;
  if (B >= 16) reinterpret_cast<uint4 *>(out)[t * (B / 16)] = r;
  if (B == 32) reinterpret_cast<uint4 *>(out)[t * 2 + 1] = make_uint4(r.w, r.z, r.y, r.x);
  if (B == 8) reinterpret_cast<uint2 *>(out)[t] = make_uint2(r.x, r.y);
}

template <class F>
void timeit(const char *name, F f, uint32_t n) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  f();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  const int R = 10;
  for (int r = 0; r < R; r++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= R;
  printf("%-36s %8.4f ms  %6.2f ns per packet per CU  %7.1f Mpps\n", name, ms, ms * 1e6 / n * 256,
         n / (ms * 1e3));
}

int main() {
  const uint32_t n = 2000000;
  uint8_t *buf;
  CK(hipMalloc(&buf, (size_t)n * SLOT));
  CK(hipMemset(buf, 0x5a, (size_t)n * SLOT));
  uint32_t *sink;
  CK(hipMalloc(&sink, (size_t)n * 4 * 4));
  uint4 *in;
  CK(hipMalloc(&in, (size_t)n * 16));
  CK(hipMemset(in, 1, (size_t)n * 16));
  uint8_t *out;
  CK(hipMalloc(&out, (size_t)n * 32));
#define FR(L, S) timeit(S ? "frames L=" #L " load+store" : "frames L=" #L " load", [&] { \
    frame_kernel<L, S><<<(n * L + 255) / 256, 256>>>(buf, sink, n); }, n)
  FR(1, false); FR(2, false); FR(4, false);
  FR(1, true); FR(2, true); FR(4, true);
  timeit("in-record 16 B load only", [&] { rec_kernel<0><<<(n + 255) / 256, 256>>>(in, out, n); }, n);
  timeit("in 16 B + out 32 B", [&] { rec_kernel<32><<<(n + 255) / 256, 256>>>(in, out, n); }, n);
  timeit("in 16 B + out 16 B", [&] { rec_kernel<16><<<(n + 255) / 256, 256>>>(in, out, n); }, n);
  timeit("in 16 B + out 8 B", [&] { rec_kernel<8><<<(n + 255) / 256, 256>>>(in, out, n); }, n);
  return 0;
}

// Microbenchmark of the memory shapes of the per-packet kernel (diagnostic,
// not product): frames of 60 B at +96 in 160-B slots, 16-B in-records, 32-B
// out-records, 2M packets.  Each pattern is timed with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct In { uint32_t off; uint16_t len; uint16_t iif; uint32_t flags; uint32_t vni; };
struct Out { uint32_t a, b, c, d, e, f, g, h; };

template <int P, int NDEP>
__global__ void __launch_bounds__(128) kern(const uint8_t *__restrict__ tbl, uint32_t tmask, uint8_t *__restrict__ buf,
                                            const In *__restrict__ in, Out *__restrict__ out, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[128 * 24];
  uint32_t i = blockIdx.x * 128 + threadIdx.x;
  if (i >= n) return;
  In p = in[i];
  uint32_t acc = p.off;
  uint32_t *w = lds + threadIdx.x * 24;
  if (P >= 1) {
    const uint4 *src = reinterpret_cast<const uint4 *>(buf + (p.off & ~15u));
    int nc = ((p.off & 15) + p.len + 15) >> 4;
    for (int c = 0; c < nc && c < 6; c++) { uint4 q = src[c]; w[4*c] = q.x; w[4*c+1] = q.y; w[4*c+2] = q.z; w[4*c+3] = q.w; }
    for (int k = 0; k < 15; k++) acc += w[k];
  }
  if (P == 2) {  // narrow field stores like a header patch
    uint8_t *q = buf + p.off;
    for (int k = 0; k < 6; k++) *reinterpret_cast<uint16_t *>(q + 2 * k) = (uint16_t)(acc + k);
    q[22] = (uint8_t)acc;
    *reinterpret_cast<uint16_t *>(q + 24) = (uint16_t)acc;
    *reinterpret_cast<uint16_t *>(q + 26) = (uint16_t)acc; *reinterpret_cast<uint16_t *>(q + 28) = (uint16_t)acc;
    *reinterpret_cast<uint16_t *>(q + 30) = (uint16_t)acc; *reinterpret_cast<uint16_t *>(q + 32) = (uint16_t)acc;
    *reinterpret_cast<uint16_t *>(q + 34) = (uint16_t)acc; *reinterpret_cast<uint16_t *>(q + 36) = (uint16_t)acc;
    *reinterpret_cast<uint16_t *>(q + 40) = (uint16_t)acc;
  }
  if (P == 3) {  // whole-chunk write-back from the LDS copy
    uint4 *dst = reinterpret_cast<uint4 *>(buf + (p.off & ~15u));
    int nc = ((p.off & 15) + p.len + 15) >> 4;
    w[3] ^= acc;
    for (int c = 0; c < nc && c < 6; c++) dst[c] = make_uint4(w[4*c], w[4*c+1], w[4*c+2], w[4*c+3]);
  }
  if (NDEP > 0) {  // dependent random loads
    uint32_t h = acc * 2654435761u;
    for (int k = 0; k < NDEP; k++) {
      uint32_t v = reinterpret_cast<const uint32_t *>(tbl)[(h >> 2) & (tmask >> 2)];
      h = (h ^ v) * 2654435761u + k;
    }
    acc ^= h;
  }
  Out o; o.a = acc; o.b = p.len; o.c = p.iif; o.d = 0; o.e = 1; o.f = 2; o.g = 3; o.h = 4;
  out[i] = o;
}

template <int P, int NDEP>
float run(const char *name, const uint8_t *tbl, uint32_t tmask, uint8_t *buf, const In *in, Out *out, uint32_t n) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++) kern<P, NDEP><<<(n + 127) / 128, 128>>>(tbl, tmask, buf, in, out, n);
  CK(hipEventRecord(a));
  const int R = 20;
  for (int r = 0; r < R; r++) kern<P, NDEP><<<(n + 127) / 128, 128>>>(tbl, tmask, buf, in, out, n);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= R;
  printf("%-34s %8.4f ms  %8.1f Mpps\n", name, ms, n / ms / 1e3);
  return ms;
}

int main(int argc, char **argv) {
  const uint32_t n = 2000000;
  const uint32_t slot = argc > 1 ? atoi(argv[1]) : 160, hr = argc > 2 ? atoi(argv[2]) : 96;
  printf("slot %u headroom %u\n", slot, hr);
  std::vector<In> hin(n);
  for (uint32_t i = 0; i < n; i++) hin[i] = In{i * slot + hr, 60, 1, 0, 1000};
  uint8_t *buf; In *din; Out *dout; uint8_t *t64, *t1;
  CK(hipMalloc(&buf, (size_t)n * slot + 256)); CK(hipMemset(buf, 0x5a, (size_t)n * slot + 256));
  CK(hipMalloc(&din, n * sizeof(In))); CK(hipMemcpy(din, hin.data(), n * sizeof(In), hipMemcpyHostToDevice));
  CK(hipMalloc(&dout, n * sizeof(Out)));
  CK(hipMalloc(&t64, 64u << 20)); CK(hipMemset(t64, 1, 64u << 20));
  CK(hipMalloc(&t1, 1u << 20)); CK(hipMemset(t1, 1, 1u << 20));
  run<0, 0>("P0 in+out records", t64, (64u << 20) - 1, buf, din, dout, n);
  run<1, 0>("P1 +window load", t64, (64u << 20) - 1, buf, din, dout, n);
  run<2, 0>("P2 +narrow patch stores", t64, (64u << 20) - 1, buf, din, dout, n);
  run<3, 0>("P3 +chunk write-back", t64, (64u << 20) - 1, buf, din, dout, n);
  run<1, 1>("P1 + 1 dep load 64MB", t64, (64u << 20) - 1, buf, din, dout, n);
  run<1, 4>("P1 + 4 dep loads 64MB", t64, (64u << 20) - 1, buf, din, dout, n);
  run<1, 10>("P1 + 10 dep loads 64MB", t64, (64u << 20) - 1, buf, din, dout, n);
  run<1, 10>("P1 + 10 dep loads 1MB", t1, (1u << 20) - 1, buf, din, dout, n);
  run<1, 30>("P1 + 30 dep loads 1MB", t1, (1u << 20) - 1, buf, din, dout, n);
  run<1, 30>("P1 + 30 dep loads 64MB", t64, (64u << 20) - 1, buf, din, dout, n);
  return 0;
}

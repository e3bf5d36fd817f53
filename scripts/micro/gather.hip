// Microbenchmark: cost of per-lane random dword gathers (diagnostic, not
// product).  Table filled with random indices so every load depends on the
// previous one; 2M lanes; table size and chain length vary.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int NDEP, int MODE>
__global__ void __launch_bounds__(256) kern(const uint32_t *__restrict__ tbl, uint32_t mask, uint32_t *__restrict__ out, uint32_t n) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (i * 2654435761u) & mask;
  if (MODE == 1) h = (blockIdx.x * 977u) & mask;            // wave-uniform address
  if (MODE == 2) h = ((i >> 3) * 2654435761u) & mask;       // 8 lanes share a line-ish
  uint32_t acc = 0;
#pragma unroll 1
  for (int k = 0; k < NDEP; k++) {
    uint32_t v = tbl[h];
    acc += v;
    h = MODE == 1 ? ((v + blockIdx.x) & mask) & ~63u : (v ^ (MODE == 2 ? (i >> 3) : i)) & mask;
  }
  out[i] = acc;
}

template <int NDEP, int MODE>
void run(const char *name, const uint32_t *t, uint32_t mask, uint32_t *out, uint32_t n) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 2; w++) kern<NDEP, MODE><<<(n + 255) / 256, 256>>>(t, mask, out, n);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  const int R = 10;
  for (int r = 0; r < R; r++) kern<NDEP, MODE><<<(n + 255) / 256, 256>>>(t, mask, out, n);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= R;
  double per = ms * 1e6 / ((double)n / 64 * NDEP) * 256;  // ns per wave-load per CU
  printf("%-28s mask %9u  %8.4f ms  %7.1f ns per wave-load per CU\n", name, mask + 1, ms, per);
}

int main() {
  const uint32_t n = 2000000;
  uint32_t *out; CK(hipMalloc(&out, n * 4));
  for (uint32_t mb : {1u, 8u, 64u, 512u}) {
    uint32_t words = mb << 18;
    std::vector<uint32_t> h(words);
    uint64_t s = 88172645463325252ull;
    for (auto &x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)s & (words - 1); }
    uint32_t *t; CK(hipMalloc(&t, words * 4ull)); CK(hipMemcpy(t, h.data(), words * 4ull, hipMemcpyHostToDevice));
    printf("table %u MB\n", mb);
    run<1, 0>("random 1 dep", t, words - 1, out, n);
    run<8, 0>("random 8 dep", t, words - 1, out, n);
    run<32, 0>("random 32 dep", t, words - 1, out, n);
    run<32, 2>("8-lane groups 32 dep", t, words - 1, out, n);
    run<32, 1>("wave-uniform 32 dep", t, words - 1, out, n);
    CK(hipFree(t));
  }
  return 0;
}

// Microbenchmark (diagnostic, not product): price of one dependent lookup
// step by access shape, to calibrate the packet kernel's table layouts.
// 2M lanes, chains of 32 dependent steps; each step loads W bytes per lane
// from a record chosen by the previous step's value.  Shapes:
//   W  = 4, 16, 32, 64 bytes per lane per step (1, 1, 2, 4 load instructions)
//   G  = lanes sharing one record (1 = fully divergent, 4, 16, 64 = uniform)
// Reported: ns of one CU per (wave, step) and per lane-step; run under
// rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum to price each
// shape in TCP accesses and TD cycles.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int STEPS = 32;

template <int W, int G>
__global__ void __launch_bounds__(256) step_kernel(const uint4 *__restrict__ tbl, uint32_t mask,
                                                   uint32_t *__restrict__ out, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t grp = i / G;
  uint32_t h = (grp * 2654435761u) & mask;  // record index (64-byte records)
  uint32_t acc = 0;
#pragma unroll 1
  for (int k = 0; k < STEPS; k++) {
    const uint4 *r = tbl + 4 * (uint64_t)h;
    uint32_t v;
    if (W == 4) {
      v = reinterpret_cast<const uint32_t *>(r)[(G >= 4) ? (i & 3) : 0];
    } else if (W == 16) {
      const uint4 q = r[(G >= 4) ? (i & 3) : 0];
      v = q.x ^ q.y ^ q.z ^ q.w;
    } else if (W == 32) {
      const uint4 a = r[0], b = r[1];
      v = a.x ^ a.y ^ b.z ^ b.w;
    } else {
      const uint4 a = r[0], b = r[1], c = r[2], d = r[3];
      v = a.x ^ b.y ^ c.z ^ d.w;
    }
    acc += v;
    h = (v ^ grp) & mask;
  }
  out[i] = acc;
}

// Occupancy sweep: one-wave blocks, dynamic LDS sized so that N waves fit
// per SIMD (160 KiB per CU / (4 N) per block); W16 G1 steps.
__global__ void __launch_bounds__(64) occ_kernel(const uint4 *__restrict__ tbl, uint32_t mask,
                                                 uint32_t *__restrict__ out, uint32_t n) {
  extern __shared__ uint32_t pad[];
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (i * 2654435761u) & mask;
  uint32_t acc = 0;
#pragma unroll 1
  for (int k = 0; k < STEPS; k++) {
    const uint4 q = tbl[4 * (uint64_t)h];
    const uint32_t v = q.x ^ q.y ^ q.z ^ q.w;
    acc += v;
    h = (v ^ i) & mask;
  }
  if (acc == 0x12345678u) pad[threadIdx.x] = acc;
  out[i] = acc;
}

void run_occ(int waves, const uint4 *t, uint32_t mask, uint32_t *out, uint32_t n) {
  const size_t lds = (160u * 1024u) / (4u * waves) - 256;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 2; w++) occ_kernel<<<(n + 63) / 64, 64, lds>>>(t, mask, out, n);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  const int R = 5;
  for (int r = 0; r < R; r++) occ_kernel<<<(n + 63) / 64, 64, lds>>>(t, mask, out, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= R;
  printf("occupancy %d waves/SIMD (W16 G1)      %8.4f ms  %7.1f ns/(wave-step) per CU\n", waves, ms,
         ms * 1e6 / ((double)n / 64 * STEPS) * 256);
}

template <int W, int G>
void run(const char *name, const uint4 *t, uint32_t mask, uint32_t *out, uint32_t n) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 2; w++) step_kernel<W, G><<<(n + 255) / 256, 256>>>(t, mask, out, n);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  const int R = 5;
  for (int r = 0; r < R; r++) step_kernel<W, G><<<(n + 255) / 256, 256>>>(t, mask, out, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= R;
  const double wave_steps = (double)n / 64 * STEPS;
  printf("%-34s %8.4f ms  %7.1f ns/(wave-step) per CU  %6.3f ns/(lane-step) per CU\n", name, ms,
         ms * 1e6 / wave_steps * 256, ms * 1e6 / ((double)n * STEPS) * 256);
}

int main() {
  const uint32_t n = 2000000;
  uint32_t *out;
  CK(hipMalloc(&out, n * 4));
  for (uint32_t mb : {1u, 2u, 4u, 8u, 16u, 64u}) {
    const uint32_t recs = mb << 14;  // 64-byte records
    std::vector<uint32_t> h((size_t)recs * 16);
    uint64_t s = 88172645463325252ull;
    for (auto &x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)s; }
    uint4 *t;
    CK(hipMalloc(&t, h.size() * 4));
    CK(hipMemcpy(t, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    printf("table %u MB\n", mb);
    if (mb != 1 && mb != 64) {
      run<16, 1>("W16 G1  (divergent dwordx4)", t, recs - 1, out, n);
      CK(hipFree(t));
      continue;
    }
    run<4, 1>("W4  G1  (divergent dword)", t, recs - 1, out, n);
    run<16, 1>("W16 G1  (divergent dwordx4)", t, recs - 1, out, n);
    run<32, 1>("W32 G1  (divergent 2x dwordx4)", t, recs - 1, out, n);
    run<64, 1>("W64 G1  (divergent 4x dwordx4)", t, recs - 1, out, n);
    run<4, 4>("W4  G4  (4 lanes / record)", t, recs - 1, out, n);
    run<16, 4>("W16 G4  (4 lanes x 16B = 1 record)", t, recs - 1, out, n);
    run<64, 4>("W64 G4  (4 lanes same 64B)", t, recs - 1, out, n);
    run<16, 16>("W16 G16", t, recs - 1, out, n);
    run<16, 64>("W16 G64 (wave-uniform)", t, recs - 1, out, n);
    for (int w : {1, 2, 3, 4, 6, 8}) run_occ(w, t, recs - 1, out, n);
    CK(hipFree(t));
  }
  return 0;
}

// Micro test: lock-free stack pushes (64-bit CAS on (tag << 32 | record)) from
// a whole grid onto a few heads, as dp_nat_prep files NAT records; then counts
// the records reachable from the heads.  Diagnostic, not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned long long ull;
__global__ void push_k(ull *head, ull *next, uint32_t n, uint32_t nheads, uint32_t tagv, int mode) {
  const uint32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
  if (rec >= n) return;
  const uint32_t h = (rec * 2654435761u) % nheads;
  const ull tag = (ull)tagv << 32;
  ull old = mode ? __hip_atomic_load(&head[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : head[h];
  for (;;) {
    const uint32_t prev = (old >> 32) == tagv ? (uint32_t)old : 0xffffffffu;
    next[rec] = ((ull)rec << 32) | prev;
    const ull got = atomicCAS(&head[h], old, tag | rec);
    if (got == old) break;
    old = got;
  }
}
int main() {
  const uint32_t n = 1 << 16;
  for (int mode = 0; mode < 2; mode++)
    for (uint32_t nheads : {563u, 4096u, 60000u}) {
      ull *head, *next;
      hipMalloc(&head, sizeof(ull) * nheads);
      hipMalloc(&next, sizeof(ull) * n);
      hipMemset(head, 0, sizeof(ull) * nheads);
      hipLaunchKernelGGL(push_k, dim3((n + 255) / 256), dim3(256), 0, 0, head, next, n, nheads, 1u, mode);
      hipDeviceSynchronize();
      std::vector<ull> h(nheads), nx(n);
      hipMemcpy(h.data(), head, sizeof(ull) * nheads, hipMemcpyDeviceToHost);
      hipMemcpy(nx.data(), next, sizeof(ull) * n, hipMemcpyDeviceToHost);
      size_t seen = 0;
      for (uint32_t e = 0; e < nheads; e++) {
        if ((h[e] >> 32) != 1) continue;
        uint32_t r = (uint32_t)h[e];
        while (r != 0xffffffffu && seen <= n) { seen++; r = (uint32_t)nx[r]; }
      }
      printf("mode %d heads %6u: reachable %zu of %u%s\n", mode, nheads, seen, n, seen == n ? "" : "  <-- LOST");
      hipFree(head);
      hipFree(next);
    }
  return 0;
}

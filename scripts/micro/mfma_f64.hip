// FP64 MFMA on gfx950: issue cost of v_mfma_f64_16x16x4_f64 and whether FP64 VALU FMAs
// of the same wave overlap it (separate pipes).  One wave per SIMD (4 waves per block).
//   K = 0: 4 independent MFMA accumulators, no VALU
//   K = 1: 8 independent v_fma_f64 streams, no MFMA (the sweep's VALU reference)
//   K = 2..5: per step one MFMA (round-robin over 4 accumulators) + 2 / 4 / 8 / 16 VALU FMAs
// Prints cycles per step; overlap shows as time ~ max(MFMA, VALU) instead of the sum.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int REP = 256;
#define F(v) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v) : "v"(a), "v"(b));
#define M(c) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);

template <int K>
__global__ void bench(long long* out, double seed) {
  double a = 0.999 + seed * 1e-9, b = 1e-3;
  d4 c0 = {seed, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double v0 = seed, v1 = seed + 1, v2 = seed + 2, v3 = seed + 3, v4 = seed + 4, v5 = seed + 5,
         v6 = seed + 6, v7 = seed + 7;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < REP; ++i) {
    if constexpr (K == 0) { M(c0) M(c1) M(c2) M(c3) }
    if constexpr (K == 1) { F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7) }
    if constexpr (K == 2) { M(c0) F(v0) F(v1) M(c1) F(v2) F(v3) M(c2) F(v4) F(v5) M(c3) F(v6) F(v7) }
    if constexpr (K == 3) {
      M(c0) F(v0) F(v1) F(v2) F(v3) M(c1) F(v4) F(v5) F(v6) F(v7)
      M(c2) F(v0) F(v1) F(v2) F(v3) M(c3) F(v4) F(v5) F(v6) F(v7)
    }
    if constexpr (K == 4) {
      M(c0) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
      M(c1) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
      M(c2) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
      M(c3) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
    }
    if constexpr (K == 5) {
      M(c0) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
      M(c1) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
      M(c2) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
      M(c3) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7) F(v0) F(v1) F(v2) F(v3) F(v4) F(v5) F(v6) F(v7)
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    out[2 * (threadIdx.x >> 6)] = t0;
    out[2 * (threadIdx.x >> 6) + 1] = t1;
  }
  const double s = c0.x + c1.y + c2.z + c3.w + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
  if (s == 12345.678) out[0] = 0;
}

int main() {
  const char* names[] = {"4 MFMA", "8 FMA", "4 MFMA + 8 FMA", "4 MFMA + 16 FMA",
                         "4 MFMA + 32 FMA", "4 MFMA + 64 FMA"};
  long long* d;
  if (hipMalloc(&d, 8 * 64) != hipSuccess) return 1;
  for (int K = 0; K < 6; ++K) {
    auto run = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, d, 1.0);
      hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, d, 1.0);
    };
    switch (K) {
      case 0: run(bench<0>); break; case 1: run(bench<1>); break; case 2: run(bench<2>); break;
      case 3: run(bench<3>); break; case 4: run(bench<4>); break; case 5: run(bench<5>); break;
    }
    long long h[8];
    if (hipMemcpy(h, d, sizeof(long long) * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    long long a = h[0], b = h[1];
    for (int w = 0; w < 4; ++w) { a = h[2 * w] < a ? h[2 * w] : a; b = h[2 * w + 1] > b ? h[2 * w + 1] : b; }
    printf("%-18s: %.1f cycles per step (1 wave per SIMD)\n", names[K], (double)(b - a) / REP);
  }
  return 0;
}

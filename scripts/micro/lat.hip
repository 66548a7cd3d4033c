// Latency microbenchmark (one wave): cycles per dependent operation on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#define AS_LDS __attribute__((address_space(3)))
#define AS_CST __attribute__((address_space(4)))
constexpr int REP = 256;
__device__ __forceinline__ long long now() { return (long long)__builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ void fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
struct KP { double a[64]; };
__global__ void lat(const KP* kp, double* out, long long* cyc, double seed) {
  __shared__ double sh[1024];
  const int lane = threadIdx.x;
  AS_LDS double* L = (AS_LDS double*)sh;
  for (int i = lane; i < 1024; i += 64) L[i] = (i * 7 % 1024) ;  // index chain
  fence();
  double x = seed + lane * 1e-3, acc = 0;
  long long t0, t1;
  // (1) dependent f64 fma
  t0 = now();
  for (int i = 0; i < REP; ++i) x = fma(x, 0.999999, 1e-7);
  fence(); t1 = now(); if (lane == 0) cyc[0] = (t1 - t0); acc += x;
  // (2) dependent ds_read_b64 (pointer chase)
  double idx = (double)lane;
  t0 = now();
  for (int i = 0; i < REP; ++i) { idx = L[(int)idx & 1023]; }
  fence(); t1 = now(); if (lane == 0) cyc[1] = (t1 - t0); acc += idx;
  // (3) f64 exp dependent
  x = 0.1 + lane * 1e-4;
  t0 = now();
  for (int i = 0; i < REP; ++i) x = exp(x) * 1e-3 + 0.05;
  fence(); t1 = now(); if (lane == 0) cyc[2] = (t1 - t0); acc += x;
  // (4) dpp f64 dependent (xor1) add
  x = lane;
  t0 = now();
  for (int i = 0; i < REP; ++i) x = x * 0.5 + dpp<0xB1>(x);
  fence(); t1 = now(); if (lane == 0) cyc[3] = (t1 - t0); acc += x;
  // (5) readlane f64 dependent
  x = lane;
  t0 = now();
  for (int i = 0; i < REP; ++i) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, 3), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), 3);
    x = __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo) * 0.5 + lane;
  }
  fence(); t1 = now(); if (lane == 0) cyc[4] = (t1 - t0); acc += x;
  // (6) dependent s_load from constant memory (index chain through kp)
  const AS_CST KP* K = (const AS_CST KP*)kp;
  int j = 0;
  t0 = now();
  for (int i = 0; i < REP; ++i) { j = __builtin_amdgcn_readfirstlane((int)K->a[j & 63] & 63); }
  t1 = now(); if (lane == 0) cyc[5] = (t1 - t0); acc += j;
  // (7) LDS write then fence then read (store->load round trip)
  t0 = now();
  for (int i = 0; i < REP; ++i) { L[lane] = x; fence(); x = L[(lane + 1) & 63] + 1.0; }
  fence(); t1 = now(); if (lane == 0) cyc[6] = (t1 - t0); acc += x;
  // (8) f64 sqrt dependent
  x = 2.0 + lane;
  t0 = now();
  for (int i = 0; i < REP; ++i) x = sqrt(x) + 1.0;
  fence(); t1 = now(); if (lane == 0) cyc[7] = (t1 - t0); acc += x;
  // (9) f64 division dependent
  x = 2.0 + lane;
  t0 = now();
  for (int i = 0; i < REP; ++i) x = 1.0 / x + 1.0;
  fence(); t1 = now(); if (lane == 0) cyc[8] = (t1 - t0); acc += x;
  // (10) 8 independent ds_read_b64 then use (gather pattern), repeated dependent via address
  t0 = now();
  int a0 = lane;
  for (int i = 0; i < REP; ++i) {
    double s = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) s += L[(a0 + w * 64) & 1023];
    a0 = ((int)s & 7) + lane;
  }
  fence(); t1 = now(); if (lane == 0) cyc[9] = (t1 - t0); acc += a0;
  // (11) s_sleep(1)+LDS poll roundtrip cost (just s_sleep)
  t0 = now();
  for (int i = 0; i < REP; ++i) __builtin_amdgcn_s_sleep(1);
  t1 = now(); if (lane == 0) cyc[10] = (t1 - t0);
  // (12) f64 add dependent
  x = lane;
  t0 = now();
  for (int i = 0; i < REP; ++i) x = x + 1e-3;
  fence(); t1 = now(); if (lane == 0) cyc[11] = (t1 - t0); acc += x;
  out[lane] = acc;
}
int main() {
  KP h; for (int i = 0; i < 64; ++i) h.a[i] = (i * 5 + 3) % 64;
  KP* d; double* o; long long* c;
  hipMalloc(&d, sizeof(KP)); hipMalloc(&o, 64 * 8); hipMalloc(&c, 16 * 8);
  hipMemcpy(d, &h, sizeof(KP), hipMemcpyHostToDevice);
  long long hc[16];
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, d, o, c, 0.3);
    hipDeviceSynchronize();
  }
  hipMemcpy(hc, c, 16 * 8, hipMemcpyDeviceToHost);
  const char* nm[] = {"fma_f64 dep", "ds_read_b64 chase", "exp_f64 dep", "dpp f64 +", "readlane f64", "s_load chase",
                      "lds st->fence->ld", "sqrt_f64 dep", "div_f64 dep", "8x ds_read sum", "s_sleep(1)", "add_f64 dep"};
  for (int i = 0; i < 12; ++i) printf("%-20s %7.1f cycles/op\n", nm[i], hc[i] / (double)REP);
  return 0;
}

// Issue-rate microbenchmark (gfx950): cycles per wave64 instruction for 8
// independent streams of one opcode, 1 wave per SIMD (4 waves per workgroup).
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int REP = 512;
#define BODY8(OP) OP(v0) OP(v1) OP(v2) OP(v3) OP(v4) OP(v5) OP(v6) OP(v7)
#define FMA(v) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v) : "v"(a), "v"(b));
#define MUL(v) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(v) : "v"(a));
#define RCP(v) asm volatile("v_rcp_f64 %0, %0" : "+v"(v));
#define RND(v) asm volatile("v_rndne_f64 %0, %0" : "+v"(v));
#define LDX(v) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(v) : "v"(k));
#define CVT(v) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(iv) : "v"(v)); asm volatile("" :: "v"(iv));
#define CND(v) { int t_; asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(t_) : "v"(k), "v"(iv)); asm volatile("" :: "v"(t_)); }
#define MOV(v) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(iv) : "v"(k)); asm volatile("" :: "v"(iv));
#define ADD(v) asm volatile("v_add_f64 %0, %0, %1" : "+v"(v) : "v"(a));
#define FMA2(v) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v) : "v"(a), "v"(b)); asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(u##v) : "v"(a), "v"(b));
#define FMA1(v) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v0) : "v"(a), "v"(b));
#define FMA4(v) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v0) : "v"(a), "v"(b)); asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v1) : "v"(a), "v"(b)); asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v2) : "v"(a), "v"(b)); asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v3) : "v"(a), "v"(b));
#define PKF(v) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(w) : "v"(w2), "v"(w3));

template <int K>
__global__ void rate(long long* out, double seed) {
  double v0 = seed, v1 = seed + 1, v2 = seed + 2, v3 = seed + 3, v4 = seed + 4, v5 = seed + 5,
         v6 = seed + 6, v7 = seed + 7, a = 0.999, b = 1e-3;
  double uv0 = seed + 8, uv1 = seed + 9, uv2 = seed + 10, uv3 = seed + 11, uv4 = seed + 12,
         uv5 = seed + 13, uv6 = seed + 14, uv7 = seed + 15;
  int k = 1, iv = 0;
  long long w = 1, w2 = 2, w3 = 3;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < REP; ++i) {
    if constexpr (K == 0) { BODY8(FMA) }
    if constexpr (K == 1) { BODY8(MUL) }
    if constexpr (K == 2) { BODY8(RCP) }
    if constexpr (K == 3) { BODY8(RND) }
    if constexpr (K == 4) { BODY8(LDX) }
    if constexpr (K == 5) { BODY8(CVT) }
    if constexpr (K == 6) { BODY8(CND) }
    if constexpr (K == 7) { BODY8(MOV) }
    if constexpr (K == 8) { BODY8(ADD) }
    if constexpr (K == 9) { BODY8(PKF) }
    if constexpr (K == 10) { BODY8(FMA2) }
    if constexpr (K == 11) { BODY8(FMA1) }
    if constexpr (K == 12) { FMA4(x) FMA4(x) }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    out[2 * (threadIdx.x >> 6)] = t0;
    out[2 * (threadIdx.x >> 6) + 1] = t1;
  }
  if (v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + iv + w + uv0 + uv1 + uv2 + uv3 + uv4 + uv5 + uv6 + uv7 == 12345.678) out[0] = 0;
}

int main() {
  const char* names[] = {"fma_f64", "mul_f64", "rcp_f64", "rndne_f64", "ldexp_f64", "cvt_i32_f64",
                         "cndmask_b32", "mov_dpp", "add_f64", "pk_fma_f32", "fma16strm", "fma1strm", "fma4strm"};
  long long* d;
  hipMalloc(&d, 8 * 64);  // 16 waves x {start, end}
  for (int K = 0; K < 13; ++K) {
    for (int waves = 1; waves <= 4; ++waves) {
      auto run = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64 * 4 * waves), 0, 0, d, 1.0);
        hipLaunchKernelGGL(kern, dim3(1), dim3(64 * 4 * waves), 0, 0, d, 1.0);
      };
      switch (K) {
        case 0: run(rate<0>); break; case 1: run(rate<1>); break; case 2: run(rate<2>); break;
        case 3: run(rate<3>); break; case 4: run(rate<4>); break; case 5: run(rate<5>); break;
        case 6: run(rate<6>); break; case 7: run(rate<7>); break; case 8: run(rate<8>); break;
        case 9: run(rate<9>); break; case 10: run(rate<10>); break;
        case 11: run(rate<11>); break; case 12: run(rate<12>); break;
      }
      long long h[32];
      hipMemcpy(h, d, sizeof(long long) * 8 * waves, hipMemcpyDeviceToHost);
      long long a = h[0], b = h[1];
      for (int w = 0; w < 4 * waves; ++w) { a = h[2 * w] < a ? h[2 * w] : a; b = h[2 * w + 1] > b ? h[2 * w + 1] : b; }
      printf("%-12s waves/SIMD=%d: %.2f cycles per wave-instruction per SIMD\n", names[K], waves,
             (double)(b - a) / (REP * (K == 10 ? 16.0 : 8.0) * waves));
    }
  }
  return 0;
}

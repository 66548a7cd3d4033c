// Counter-based Philox4x32-10 (Salmon et al., SC'11) with *addressable* draws.
//
// Stan seeds one boost::ecuyer1988 stream per chain and consumes it
// sequentially.  A lock-stepped device sampler cannot share a sequential
// stream layout with anything else, so every random number here is addressed
// by (key = seed x global chain id, counter = purpose tag x iteration x index).
// The CPU oracle (oracle/fitoct_oracle.c) addresses the same numbers, which
// makes GPU and CPU trajectories comparable draw by draw.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define FITOCT_HD __host__ __device__ __forceinline__
#else
#define FITOCT_HD static inline
#endif

namespace fitoct {

enum RngTag : uint32_t {
  TAG_INIT = 1,    // c0 = init attempt, c2 = param index
  TAG_SSMOM = 2,   // c0 = step-size search index, c2 = param pair, c3 = trial
  TAG_MOM = 3,     // c0 = iteration, c2 = param pair
  TAG_DIR = 4,     // c0 = iteration, c2 = tree depth
  TAG_TOP = 5,     // c0 = iteration, c2 = tree depth
  TAG_MERGE = 6,   // c0 = iteration, c1 = tag | level<<8 | depth<<16, c2 = leaf
};

struct U4 { uint32_t x, y, z, w; };

FITOCT_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

FITOCT_HD U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#if defined(__HIPCC__)
#pragma unroll
#endif
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
    U4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// 53-bit uniform in [0,1)
FITOCT_HD double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

struct RngKey { uint32_t k0, k1; };

FITOCT_HD RngKey make_key(uint64_t seed, uint32_t chain_gid) {
  RngKey k;
  k.k0 = (uint32_t)seed;
  k.k1 = (uint32_t)(seed >> 32) ^ (chain_gid * 0x9E3779B9u + 0x7F4A7C15u);
  return k;
}

FITOCT_HD double uniform(RngKey k, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  U4 c = {c0, c1, c2, c3};
  U4 r = philox4x32_10(c, k.k0, k.k1);
  return u53(r.x, r.y);
}

}  // namespace fitoct

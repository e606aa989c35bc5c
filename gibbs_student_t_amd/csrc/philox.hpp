// Philox4x32-10 counter-based RNG (Salmon et al., SC'11) and the variate maps built on it.
//
// Counter layout used by the sampler: (index, tag, sweep, chain) with key = seed.  Every
// draw is a pure function of (seed, chain, sweep, stage/step, index), so chains give the
// same numbers whatever the launch shape or the GPU they are sharded to.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GST_HD __host__ __device__ __forceinline__
#else
#define GST_HD inline
#endif

namespace gst {

struct u32x4 {
  uint32_t v[4];
};

GST_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

GST_HD u32x4 philox4x32_10(u32x4 ctr, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  uint32_t c0 = ctr.v[0], c1 = ctr.v[1], c2 = ctr.v[2], c3 = ctr.v[3];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32 -> 64-bit product per multiplier gives both halves (v_mad_u64_u32 on
    // gfx950, instead of separate quarter-rate v_mul_hi_u32 + v_mul_lo_u32)
    const uint64_t p0 = (uint64_t)M0 * c0, p1 = (uint64_t)M1 * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
    k0 += W0;
    k1 += W1;
  }
  u32x4 o;
  o.v[0] = c0;
  o.v[1] = c1;
  o.v[2] = c2;
  o.v[3] = c3;
  return o;
}

// 53-bit uniform in [0, 1) from two 32-bit words.
GST_HD double u01(uint32_t lo, uint32_t hi) {
  const uint64_t x = ((uint64_t)hi << 32) | (uint64_t)lo;
  return (double)(x >> 11) * 0x1.0p-53;
}

struct Rng {
  uint32_t k0, k1;      // seed
  uint32_t chain;       // global chain id (low 32 bits)
  uint32_t sweep;       // global sweep index (low 32 bits)
  GST_HD u32x4 draw(uint32_t index, uint32_t tag) const {
    u32x4 c;
    c.v[0] = index;
    c.v[1] = tag;
    c.v[2] = sweep;
    c.v[3] = chain;
    return philox4x32_10(c, k0, k1);
  }
  // two independent uniforms in [0,1)
  GST_HD void uniform2(uint32_t index, uint32_t tag, double& a, double& b) const {
    const u32x4 r = draw(index, tag);
    a = u01(r.v[0], r.v[1]);
    b = u01(r.v[2], r.v[3]);
  }
};

// Stage tags (bits 24..31) | step/attempt (bits 0..23).
enum : uint32_t {
  TAG_WHITE = 1u << 24,
  TAG_HYPER = 2u << 24,
  TAG_BDRAW = 3u << 24,
  TAG_THETA = 4u << 24,
  TAG_Z = 5u << 24,
  TAG_ALPHA = 6u << 24,
  TAG_DF = 7u << 24,
};

}  // namespace gst

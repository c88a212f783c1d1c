// Stateless counter-based dropout RNG shared by every kernel that drops
// (LayerNorm in/out dropout, attention-probability dropout, standalone dropout).
//
// keep(seed, idx) = h(idx) >= p * 2^32, where for the 64-bit element index idx = hi:lo
//   x = (lo ^ s0) * 0x9E3779B1 + (hi * 0x27D4EB ^ s1)      (an odd-multiplier bijection of lo)
//   h = lowbias32(x)                                      (xor-shift / multiply finaliser)
// and (s0, s1) are derived from the 64-bit call seed on the host (splitmix64).
//
// The mask is a pure function of (seed, element index), so the backward pass
// regenerates it instead of storing it (no mask tensor in HBM), and a debug
// entry point (ca_dropout_mask) materialises it for the PyTorch references in
// the tests.  The host picks a fresh seed per call (cloud_amd/ops/dropout.py).
//
// Cost: every element of an attention-probability matrix and of every BERT hidden
// state draws one hash per pass (forward and backward regenerate it), so the hash is
// sized for the VALU: 3 quarter-rate 32-bit multiplies + 1 full-rate 24-bit one and ~8
// single-cycle ops, against nine 32-bit multiply pieces plus 64-bit shifts for the
// splitmix64-per-element form it replaced (the attention / LayerNorm kernels were not
// bound by it: attention forward 24.2 -> 24.0 us, docs/performance.md "BERT step, round 3").
#pragma once
#include <stdint.h>

struct DropCfg {
  uint32_t s0, s1;  // per-call hash keys
  uint32_t thresh;  // drop iff hash < thresh  (thresh = p * 2^32)
  float scale;      // 1 / (1 - p)
  int on;
};

__host__ __device__ inline uint64_t ca_splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ inline DropCfg make_drop(float p, uint64_t seed) {
  DropCfg d;
  const uint64_t k = ca_splitmix64(seed);
  d.s0 = (uint32_t)k;
  d.s1 = (uint32_t)(k >> 32);
  d.on = p > 0.f;
  double t = (double)p * 4294967296.0;
  d.thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  d.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  return d;
}

__device__ __forceinline__ uint32_t ca_hash32(const DropCfg& d, uint64_t idx) {
  const uint32_t lo = (uint32_t)idx, hi = (uint32_t)(idx >> 32);
  uint32_t x = (lo ^ d.s0) * 0x9E3779B1u + (__umul24(hi, 0x27D4EBu) ^ d.s1);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// multiplier applied to element idx: 0 (dropped) or 1/(1-p) (kept)
__device__ __forceinline__ float drop_mul(const DropCfg& d, uint64_t idx) {
  return ca_hash32(d, idx) < d.thresh ? 0.f : d.scale;
}

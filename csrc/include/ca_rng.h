// Stateless counter-based dropout RNG shared by every kernel that drops
// (LayerNorm in/out dropout, attention-probability dropout, standalone dropout).
//
// keep(seed, idx) = splitmix64(seed + (idx + 1) * phi) >> 32  >=  p * 2^32
//
// The mask is a pure function of (seed, element index), so the backward pass
// regenerates it instead of storing it (no mask tensor in HBM), and a debug
// entry point (ca_dropout_mask) materialises it for the PyTorch references in
// the tests.  The host picks a fresh seed per call (cloud_amd/ops/dropout.py).
#pragma once
#include <stdint.h>

struct DropCfg {
  uint64_t seed;
  uint32_t thresh;  // drop iff hash < thresh  (thresh = p * 2^32)
  float scale;      // 1 / (1 - p)
  int on;
};

__host__ __device__ inline DropCfg make_drop(float p, uint64_t seed) {
  DropCfg d;
  d.seed = seed;
  d.on = p > 0.f;
  double t = (double)p * 4294967296.0;
  d.thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  d.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  return d;
}

__device__ __forceinline__ uint32_t ca_hash32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + (idx + 1ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// multiplier applied to element idx: 0 (dropped) or 1/(1-p) (kept)
__device__ __forceinline__ float drop_mul(const DropCfg& d, uint64_t idx) {
  return ca_hash32(d.seed, idx) < d.thresh ? 0.f : d.scale;
}

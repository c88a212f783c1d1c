// Stateless counter-based dropout RNG shared by every kernel that drops
// (LayerNorm in/out dropout, attention-probability dropout, standalone dropout).
//
// keep(seed, idx) = half_(idx & 1)(h(idx >> 1)) >= p * 2^16 -- one 32-bit hash decides TWO
// adjacent elements with its low / high 16 bits -- where for the 64-bit pair index i = hi:lo
//   x = (lo ^ s0) * 0x9E3779B1 + (hi * 0x27D4EB ^ s1)      (an odd-multiplier bijection of lo)
//   h = lowbias32(x)                                      (xor-shift / multiply finaliser)
// and (s0, s1) are derived from the 64-bit call seed on the host (splitmix64).  p is kept to
// 1/65536 (0.1 -> 0.100006).
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
// splitmix64-per-element form it replaced (attention forward 24.2 -> 24.0 us,
// docs/performance.md "BERT step, round 3").  Round 5: one hash per element PAIR (drop_mul4 for
// four consecutive elements in one thread) -- at BERT's hidden size a LayerNorm row drew 24
// hashes per lane forward and again backward, ~7 us of VALU per call at M = 8192.
#pragma once
#include <stdint.h>

struct DropCfg {
  uint32_t s0, s1;  // per-call hash keys
  uint32_t thresh;  // drop iff the element's 16-bit half-hash < thresh  (thresh = p * 2^16)
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
  const double t = (double)p * 65536.0 + 0.5;
  d.thresh = t >= 65536.0 ? 65536u : (uint32_t)t;
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
  const uint32_t h = ca_hash32(d, idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xffffu)) < d.thresh ? 0.f : d.scale;
}

// multipliers of the four elements idx .. idx + 3: two hashes (three when idx is odd)
__device__ __forceinline__ void drop_mul4(const DropCfg& d, uint64_t idx, float (&m)[4]) {
  const uint64_t i0 = idx >> 1;
  const uint32_t h0 = ca_hash32(d, i0), h1 = ca_hash32(d, i0 + 1);
  uint32_t r[4];
  if (!(idx & 1)) {
    r[0] = h0 & 0xffffu;
    r[1] = h0 >> 16;
    r[2] = h1 & 0xffffu;
    r[3] = h1 >> 16;
  } else {
    r[0] = h0 >> 16;
    r[1] = h1 & 0xffffu;
    r[2] = h1 >> 16;
    r[3] = ca_hash32(d, i0 + 2) & 0xffffu;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = r[k] < d.thresh ? 0.f : d.scale;
}

// Element pairs split over adjacent lanes (lane l holds key 2m + (l & 1) of each of its rows):
// the lane pair computes ONE hash per row pair -- the even lane row rr, the odd lane row rr + 1 --
// and swaps them (DPP quad_perm [1,0,3,2]).  pidx = this lane's (even-key) pair index for row
// rr + (lane & 1); returns the multipliers of this lane's element in rows rr and rr + 1.
__device__ __forceinline__ void drop_mul_lanepair(const DropCfg& d, uint64_t pidx, int lane, float& m0, float& m1) {
  const uint32_t h = ca_hash32(d, pidx);
  const uint32_t hx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)h, 0xb1, 0xf, 0xf, false);
  const bool odd = lane & 1;
  const uint32_t h0 = odd ? hx : h, h1 = odd ? h : hx;
  m0 = (odd ? h0 >> 16 : h0 & 0xffffu) < d.thresh ? 0.f : d.scale;
  m1 = (odd ? h1 >> 16 : h1 & 0xffffu) < d.thresh ? 0.f : d.scale;
}

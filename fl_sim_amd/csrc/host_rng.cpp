// host_rng.cpp — compat-mode RNG: the MT19937 streams the reference consumes, advanced on the host.
//
// The reference draws its stochastic-rounding uniforms from Python's global `random` module
// (compressors.py:277, 316, 349, 386) and its Rand-K permutation from numpy's global legacy
// RandomState (compressors.py:285-287, np.random.shuffle).  Both are MT19937 (Matsumoto & Nishimura
// 1998) with the same state layout: 624 words + a position.  The caller exports the interpreter's
// state (random.getstate() / np.random.get_state()), these functions advance it exactly as the
// interpreter would, and the caller writes it back — so a drop-in call leaves both global streams
// where the reference would have left them.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "flc_runtime.hpp"

namespace {

constexpr int N = 624, M = 397;

struct MT {
  uint32_t* mt;
  int32_t pos;

  void refill() {
    constexpr uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATRIX = 0x9908b0dfu;
    int k = 0;
    uint32_t y;
    for (; k < N - M; ++k) {
      y = (mt[k] & UPPER) | (mt[k + 1] & LOWER);
      mt[k] = mt[k + M] ^ (y >> 1) ^ ((y & 1u) ? MATRIX : 0u);
    }
    for (; k < N - 1; ++k) {
      y = (mt[k] & UPPER) | (mt[k + 1] & LOWER);
      mt[k] = mt[k + (M - N)] ^ (y >> 1) ^ ((y & 1u) ? MATRIX : 0u);
    }
    y = (mt[N - 1] & UPPER) | (mt[0] & LOWER);
    mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ ((y & 1u) ? MATRIX : 0u);
    pos = 0;
  }

  inline uint32_t next32() {
    if (pos >= N) refill();
    uint32_t y = mt[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  // random.random() (Modules/_randommodule.c) == numpy legacy random_sample: 53-bit res
  inline double next_double() {
    const uint32_t a = next32() >> 5, b = next32() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }

  // numpy random_interval(max) for max <= 0xffffffff: masked rejection sampling
  inline uint32_t interval(uint32_t mx) {
    if (mx == 0) return 0;
    uint32_t mask = mx;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > mx) {
    }
    return v;
  }
};

}  // namespace

extern "C" {

int flc_mt_random_doubles(uint32_t* mt_state624, int32_t* mt_pos, double* out, int64_t n) {
  if (!mt_state624 || !mt_pos || (n > 0 && !out) || n < 0)
    return flc::fail(FLC_EINVAL, "flc_mt_random_doubles: bad arguments");
  if (*mt_pos < 0 || *mt_pos > N) return flc::fail(FLC_EINVAL, "flc_mt_random_doubles: bad position");
  MT g{mt_state624, *mt_pos};
  for (int64_t i = 0; i < n; ++i) out[i] = g.next_double();
  *mt_pos = g.pos;
  return FLC_OK;
}

int flc_np_shuffle_prefix(uint32_t* mt_state624, int32_t* mt_pos, int64_t D, int64_t K, int32_t* out_idx) {
  if (!mt_state624 || !mt_pos || D < 0 || K < 0 || (K > 0 && !out_idx) || D > 0x7fffffffLL)
    return flc::fail(FLC_EINVAL, "flc_np_shuffle_prefix: bad arguments");
  if (*mt_pos < 0 || *mt_pos > N) return flc::fail(FLC_EINVAL, "flc_np_shuffle_prefix: bad position");
  MT g{mt_state624, *mt_pos};
  std::vector<int32_t> perm((size_t)D);
  for (int64_t i = 0; i < D; ++i) perm[(size_t)i] = (int32_t)i;
  // mtrand.pyx _shuffle_raw: for i in reversed(range(1, n)): j = random_interval(i); swap(i, j)
  for (int64_t i = D - 1; i >= 1; --i) {
    const uint32_t j = g.interval((uint32_t)i);
    const int32_t t = perm[(size_t)i];
    perm[(size_t)i] = perm[j];
    perm[j] = t;
  }
  const int64_t kk = K < D ? K : D;
  if (kk > 0) memcpy(out_idx, perm.data(), (size_t)kk * sizeof(int32_t));
  *mt_pos = g.pos;
  return FLC_OK;
}

}  // extern "C"

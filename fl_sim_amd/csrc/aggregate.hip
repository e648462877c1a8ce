// aggregate.hip — server-side aggregation of client deltas for gfx950
// (reference: fl_sim/nodes.py:1116-1180 add_parameters / avg_parameters / update_gradients and
//  fl_sim/algorithms/fedopt/_fedopt.py:196-265 FedOptServer.update).
//
// The reference folds messages one at a time with torch CPU `add_(other, alpha=w)`, which is exactly
// one fp32 fmaf(w, other, acc) per element per message.  weighted_sum fuses the whole fold: every
// element is read once from each of the n sources and written once, with the fmaf chain in message
// order, so the result is bit-identical to the reference's sequential loop.  HBM bytes per element:
// 4 * n_src reads + 4 read (unless init = 0) + 4 written.
//
// fedopt_step is the element-wise tail of FedOptServer.update (v update + theta update) in one pass;
// each arithmetic step is rounded exactly where torch's CPU kernels round (no contraction: the
// library is compiled with -ffp-contract=off and fmaf is written out where torch uses an fma).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "flc_device.hpp"
#include "flc_runtime.hpp"

namespace flc {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxSrc = 16;  // sources per launch; longer message lists chain launches in order

struct SrcPack {
  const float* p[kMaxSrc];
  float w[kMaxSrc];
  int n;
};

template <int INIT, bool VEC>
__global__ __launch_bounds__(kThreads) void weighted_sum_kernel(SrcPack s, int64_t n, float beta, float* __restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  if (VEC) {
    const int64_t n4 = n >> 2;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += stride) {
      float4 a;
      if (INIT == 1) {
        a = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        a = reinterpret_cast<const float4*>(dst)[i];
        if (INIT == 0) a = make_float4(a.x * beta, a.y * beta, a.z * beta, a.w * beta);
      }
      // every source's float4 loaded first (unrolled, guarded): one batch of loads in flight per thread instead of
      // one load -> fmaf round trip per message; then the fmaf chain in message order
      float4 v[kMaxSrc];
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m)
        if (m < s.n) v[m] = ld_stream(s.p[m] + 4 * i);
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m) {
        if (m < s.n) {
          const float w = s.w[m];
          a = make_float4(fmaf(w, v[m].x, a.x), fmaf(w, v[m].y, a.y), fmaf(w, v[m].z, a.z), fmaf(w, v[m].w, a.w));
        }
      }
      reinterpret_cast<float4*>(dst)[i] = a;
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    float a = INIT == 1 ? 0.0f : (INIT == 0 ? dst[i] * beta : dst[i]);
    for (int m = 0; m < s.n; ++m) a = fmaf(s.w[m], s.p[m][i], a);
    dst[i] = a;
  }
}

template <int OPT>
__global__ __launch_bounds__(kThreads) void fedopt_step_kernel(float* __restrict__ theta, const float* __restrict__ delta,
                                                               float* __restrict__ v, int64_t n, float lr, float beta2,
                                                               float one_minus_beta2, float neg_one_minus_beta2,
                                                               float tau) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float d = delta[i];
    if (OPT == FLC_OPT_AVG) {
      theta[i] = fmaf(lr, d, theta[i]);  // sp.add_(dp, alpha=lr)           _fedopt.py:232-233
      continue;
    }
    const float d2 = d * d;  // dp.pow(2)
    float vi = v[i];
    if (OPT == FLC_OPT_ADAGRAD) {
      vi = vi + d2;  // vp.add_(dp.pow(2))                             _fedopt.py:248-250
    } else if (OPT == FLC_OPT_YOGI) {
      // vp.addcmul_(d2, sign(vp - d2), value=-(1-beta2)): self + value * t1 * t2   _fedopt.py:252-258
      const float diff = vi - d2;
      const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : (diff == 0.f ? 0.f : diff));
      vi = vi + (neg_one_minus_beta2 * d2) * sg;
    } else {
      // vp.mul_(beta2).add_(dp.pow(2), alpha=1-beta2)                 _fedopt.py:260-263
      vi = fmaf(one_minus_beta2, d2, vi * beta2);
    }
    v[i] = vi;
    // sp.addcdiv_(dp, vp.sqrt() + tau, value=lr): self + value * t1 / t2   _fedopt.py:235-239
    const float den = sqrtf(vi) + tau;
    theta[i] = theta[i] + (lr * d) / den;
  }
}

// FedDRServer.update after the x_tilde fold (_feddr.py:166-190), one pass over theta, y and x_tilde:
//   y     = fmaf(alpha, theta - y, y)          yp.data.add_(mp.data - yp.data, alpha=alpha)   _feddr.py:169-170
//   t     = cx * x_til + cy * y               (coeff/eta) * xtp + (1/(N+1)) * yp            _feddr.py:184-185
//   theta = prox(t)                            regularizer.prox_eval                         _feddr.py:186-190
// prox: FLC_PROX_NONE (NullRegularizer), FLC_PROX_L1 sign(t) * clamp(|t| - pc, min=0) (L1Norm,
// regularizers.py:154-159), FLC_PROX_SCALE t * pc (L2NormSquared with pc = fp32(1/(1+2c)), regularizers.py:193-200;
// L2Norm's factor needs the global norm of t first, so the host runs NONE and then scales).  Each torch op rounds
// to fp32 on its own, so nothing here is contracted (-ffp-contract=off) except the one fmaf add_(alpha) is.
template <int PROX>
__global__ __launch_bounds__(kThreads) void feddr_combine_kernel(float* __restrict__ theta, float* __restrict__ y,
                                                                 const float* __restrict__ x_til, int64_t n,
                                                                 float alpha, float cx, float cy, float pc) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float yo = y[i];
    const float yn = fmaf(alpha, theta[i] - yo, yo);
    y[i] = yn;
    float t = cx * x_til[i] + cy * yn;
    if (PROX == FLC_PROX_L1) {
      float m = fabsf(t) - pc;
      m = m < 0.f ? 0.f : m;  // clamp(min=0) keeps NaN
      const float sg = (float)((t > 0.f) - (t < 0.f));
      t = sg * m;
    } else if (PROX == FLC_PROX_SCALE) {
      t = t * pc;
    }
    theta[i] = t;
  }
}

// ------------------------------------------------------------------------------------------------
// float64 models and messages: the reference's torch ops keep float64 tensors float64 (add_ with alpha is one fp64
// fma per element, the scalars stay Python doubles), so the same fold / step / FedDR pass run in fp64
// (flc_weighted_sum_f64, flc_fedopt_step_f64, flc_feddr_combine_f64; per tensor, two doubles per 16-B load)
// ------------------------------------------------------------------------------------------------
typedef double f64x2 __attribute__((ext_vector_type(2)));

struct SrcPack64 {
  const double* p[kMaxSrc];
  double w[kMaxSrc];
  int n;
};

template <int INIT, bool VEC>
__global__ __launch_bounds__(kThreads) void weighted_sum64_kernel(SrcPack64 s, int64_t n, double beta,
                                                                  double* __restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  if (VEC) {
    const int64_t n2 = n >> 1;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n2; i += stride) {
      double2 a;
      if (INIT == 1) {
        a = make_double2(0.0, 0.0);
      } else {
        a = reinterpret_cast<const double2*>(dst)[i];
        if (INIT == 0) a = make_double2(a.x * beta, a.y * beta);
      }
      double2 v[kMaxSrc];
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m)
        if (m < s.n) {
          const f64x2 q = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(s.p[m]) + i);
          v[m] = make_double2(q.x, q.y);
        }
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m) {
        if (m < s.n) {
          const double w = s.w[m];
          a = make_double2(fma(w, v[m].x, a.x), fma(w, v[m].y, a.y));
        }
      }
      reinterpret_cast<double2*>(dst)[i] = a;
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    double a = INIT == 1 ? 0.0 : (INIT == 0 ? dst[i] * beta : dst[i]);
    for (int m = 0; m < s.n; ++m) a = fma(s.w[m], s.p[m][i], a);
    dst[i] = a;
  }
}

template <int OPT>
__global__ __launch_bounds__(kThreads) void fedopt_step64_kernel(double* __restrict__ theta,
                                                                 const double* __restrict__ delta, double* __restrict__ v,
                                                                 int64_t n, double lr, double beta2, double omb,
                                                                 double nomb, double tau) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const double d = delta[i];
    if (OPT == FLC_OPT_AVG) {
      theta[i] = fma(lr, d, theta[i]);  // _fedopt.py:232-233
      continue;
    }
    const double d2 = d * d;
    double vi = v[i];
    if (OPT == FLC_OPT_ADAGRAD) {
      vi = vi + d2;  // _fedopt.py:248-250
    } else if (OPT == FLC_OPT_YOGI) {
      const double diff = vi - d2;  // _fedopt.py:252-258
      const double sg = diff > 0.0 ? 1.0 : (diff < 0.0 ? -1.0 : (diff == 0.0 ? 0.0 : diff));
      vi = vi + (nomb * d2) * sg;
    } else {
      vi = fma(omb, d2, vi * beta2);  // _fedopt.py:260-263
    }
    v[i] = vi;
    theta[i] = theta[i] + (lr * d) / (sqrt(vi) + tau);  // _fedopt.py:235-239
  }
}

template <int PROX>
__global__ __launch_bounds__(kThreads) void feddr_combine64_kernel(double* __restrict__ theta, double* __restrict__ y,
                                                                   const double* __restrict__ x_til, int64_t n,
                                                                   double alpha, double cx, double cy, double pc) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const double yo = y[i];
    const double yn = fma(alpha, theta[i] - yo, yo);
    y[i] = yn;
    double t = cx * x_til[i] + cy * yn;
    if (PROX == FLC_PROX_L1) {
      double m = fabs(t) - pc;
      m = m < 0.0 ? 0.0 : m;
      t = (double)((t > 0.0) - (t < 0.0)) * m;
    } else if (PROX == FLC_PROX_SCALE) {
      t = t * pc;
    }
    theta[i] = t;
  }
}

// ------------------------------------------------------------------------------------------------
// a whole model in one launch (flc_model_fold): a model's parameters are many small tensors (cnn_femmist_tiny: 8 of
// 10 .. 401,408 elements), and one fold launch + one step launch per tensor is launch-bound (~14 us each from Python).
// Block b serves one 4096-element chunk of one tensor (the tensor found from the pack's block offsets, as
// delta_flatten does); per element the fold of weighted_sum (same init, same fmaf chain in message order) and, with
// OPT >= 0, the step of fedopt_step on the folded value — the same roundings as the two kernels, in one pass.
// ------------------------------------------------------------------------------------------------
constexpr int kModelT = 16;              // tensors per launch (kernel-argument budget: ~2.7 KB)
constexpr int kModelChunk = kThreads * 4;  // elements per block: one float4 per thread, every load in flight at once

struct ModelPack {
  float* dst[kModelT];
  float* theta[kModelT];
  float* v[kModelT];
  const float* src[kMaxSrc][kModelT];
  int64_t n[kModelT];
  int blk0[kModelT + 1];
  float w[kMaxSrc];
  unsigned vec;  // bit t: tensor t's operands are 16-B aligned
  int nt, ns;
};

// opt_step: flc_device.hpp (shared with the compressed round's fold, wire.hip)
template <int INIT, int OPT>  // OPT < 0: the fold only
__global__ __launch_bounds__(kThreads) void model_fold_kernel(ModelPack p, float beta, float lr, float beta2, float omb,
                                                              float nomb, float tau) {
  const int b = blockIdx.x;
  const int t = pack_entry<kModelT>(p.blk0, p.nt, b);  // (uniform)
  float* __restrict__ dst = p.dst[t];
  const int64_t n = p.n[t];
  const int64_t c0 = (int64_t)(b - p.blk0[t]) * kModelChunk;
  const int64_t c1 = c0 + kModelChunk < n ? c0 + kModelChunk : n;
  if ((p.vec >> t) & 1u) {
    for (int64_t i = c0 + 4 * (int64_t)threadIdx.x; i < c1; i += 4 * kThreads) {
      if (i + 4 > c1) {  // the tensor's n % 4 tail
        for (int64_t e = i; e < c1; ++e) {
          float a = INIT == 1 ? 0.0f : (INIT == 0 ? dst[e] * beta : dst[e]);
          for (int m = 0; m < p.ns; ++m) a = fmaf(p.w[m], p.src[m][t][e], a);
          dst[e] = a;
          if (OPT >= 0) opt_step<OPT < 0 ? 0 : OPT>(p.theta[t][e], a, OPT > 0 ? p.v[t] + e : nullptr, lr, beta2, omb,
                                                  nomb, tau);
        }
        break;
      }
      float4 sv[kMaxSrc];
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m)
        if (m < p.ns) sv[m] = *reinterpret_cast<const float4*>(p.src[m][t] + i);
      float4 a;
      if (INIT == 1) {
        a = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        a = *reinterpret_cast<const float4*>(dst + i);
        if (INIT == 0) a = make_float4(a.x * beta, a.y * beta, a.z * beta, a.w * beta);
      }
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m) {
        if (m < p.ns) {
          const float w = p.w[m];
          a = make_float4(fmaf(w, sv[m].x, a.x), fmaf(w, sv[m].y, a.y), fmaf(w, sv[m].z, a.z), fmaf(w, sv[m].w, a.w));
        }
      }
      *reinterpret_cast<float4*>(dst + i) = a;
      if (OPT >= 0) {
        float4 th = *reinterpret_cast<const float4*>(p.theta[t] + i);
        float* vp = OPT > 0 ? p.v[t] + i : nullptr;
        opt_step<OPT < 0 ? 0 : OPT>(th.x, a.x, vp, lr, beta2, omb, nomb, tau);
        opt_step<OPT < 0 ? 0 : OPT>(th.y, a.y, OPT > 0 ? vp + 1 : nullptr, lr, beta2, omb, nomb, tau);
        opt_step<OPT < 0 ? 0 : OPT>(th.z, a.z, OPT > 0 ? vp + 2 : nullptr, lr, beta2, omb, nomb, tau);
        opt_step<OPT < 0 ? 0 : OPT>(th.w, a.w, OPT > 0 ? vp + 3 : nullptr, lr, beta2, omb, nomb, tau);
        *reinterpret_cast<float4*>(p.theta[t] + i) = th;
      }
    }
    return;
  }
  for (int64_t e = c0 + threadIdx.x; e < c1; e += kThreads) {
    float a = INIT == 1 ? 0.0f : (INIT == 0 ? dst[e] * beta : dst[e]);
    for (int m = 0; m < p.ns; ++m) a = fmaf(p.w[m], p.src[m][t][e], a);
    dst[e] = a;
    if (OPT >= 0) opt_step<OPT < 0 ? 0 : OPT>(p.theta[t][e], a, OPT > 0 ? p.v[t] + e : nullptr, lr, beta2, omb, nomb,
                                            tau);
  }
}

// avg_parameters and update_gradients of one round in ONE launch (flc_avg_and_gradients): the variance-reduced
// servers (fedprox/_fedprox.py:163-167, fedpd/_fedpd.py:197-202, proxskip/_proxskip.py:212-216,
// pfedmac/_pfedmac.py:158-162) call the two back to back over the same messages.  Entry t of the pack is a parameter
// (weights w, init 0: θ·inertia first, or 2: a chained launch continues) or a gradient (weights w2, init 1: from +0,
// or 2); per element the same fmaf chain in message order as model_fold_kernel's fold.
struct PairPack {
  float* dst[kModelT];
  const float* src[kMaxSrc][kModelT];
  int64_t n[kModelT];
  int blk0[kModelT + 1];
  float w[kMaxSrc];
  float w2[kMaxSrc];
  unsigned vec;   // bit t: entry t's operands are 16-B aligned
  unsigned grad;  // bit t: entry t is a gradient (weights w2)
  int init[kModelT];
  int nt, ns;
};

__global__ __launch_bounds__(kThreads) void pair_fold_kernel(PairPack p, float beta) {
  const int b = blockIdx.x;
  const int t = pack_entry<kModelT>(p.blk0, p.nt, b);  // (uniform)
  float* __restrict__ dst = p.dst[t];
  const int64_t n = p.n[t];
  const int64_t c0 = (int64_t)(b - p.blk0[t]) * kModelChunk;
  const int64_t c1 = c0 + kModelChunk < n ? c0 + kModelChunk : n;
  const int init = p.init[t];
  const float* __restrict__ w = ((p.grad >> t) & 1u) ? p.w2 : p.w;
  if ((p.vec >> t) & 1u) {
    for (int64_t i = c0 + 4 * (int64_t)threadIdx.x; i < c1; i += 4 * kThreads) {
      if (i + 4 > c1) {  // the tensor's n % 4 tail
        for (int64_t e = i; e < c1; ++e) {
          float a = init == 1 ? 0.0f : (init == 0 ? dst[e] * beta : dst[e]);
          for (int m = 0; m < p.ns; ++m) a = fmaf(w[m], p.src[m][t][e], a);
          dst[e] = a;
        }
        break;
      }
      float4 sv[kMaxSrc];
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m)
        if (m < p.ns) sv[m] = *reinterpret_cast<const float4*>(p.src[m][t] + i);
      float4 a;
      if (init == 1) {
        a = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        a = *reinterpret_cast<const float4*>(dst + i);
        if (init == 0) a = make_float4(a.x * beta, a.y * beta, a.z * beta, a.w * beta);
      }
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m) {
        if (m < p.ns) {
          const float wm = w[m];
          a = make_float4(fmaf(wm, sv[m].x, a.x), fmaf(wm, sv[m].y, a.y), fmaf(wm, sv[m].z, a.z), fmaf(wm, sv[m].w, a.w));
        }
      }
      *reinterpret_cast<float4*>(dst + i) = a;
    }
    return;
  }
  for (int64_t e = c0 + threadIdx.x; e < c1; e += kThreads) {
    float a = init == 1 ? 0.0f : (init == 0 ? dst[e] * beta : dst[e]);
    for (int m = 0; m < p.ns; ++m) a = fmaf(w[m], p.src[m][t][e], a);
    dst[e] = a;
  }
}

// FedDyn / pFedMe server updates on a whole model in one pass (flc_model_fold_server), the model pack as in
// model_fold_kernel with `theta` holding the second per-element state (FedDyn's h, pFedMe's saved θ):
//   KIND 1 FedDyn (feddyn/_feddyn.py:172-184): per message m in order h = fmaf(c, fl(src_m - θ0), h)
//          (hp.add_(mp - p, alpha=-mu/N) with the model still at θ0); FOLD: θ = the avg fold of θ0 (INIT 0: θ0 * beta
//          first, avg_parameters' mul_(inertia)), line 184's p.add(...) is dropped by the reference (no effect);
//   KIND 2 pFedMe (pfedme/_pfedme.py:166-175): FOLD: a = the avg fold of θ0 (INIT 0, or INIT 2 with no message:
//          avg_parameters returns early), then θ = fmaf(c2, θ0, fl(a * c)) (mul_(beta).add_(prev, alpha=1-beta));
//          !FOLD (more messages than one launch folds: the fold ran in chained model_fold launches, θ0 saved in
//          `theta`): θ = fmaf(c2, saved, fl(θ * c)).
// Every step rounds where the reference's torch CPU ops round (add_(alpha) is one fma, mul_ and the subtraction one
// rounding each); nothing else is contracted (-ffp-contract=off).
template <int KIND, bool FOLD, int INIT>
__device__ __forceinline__ float server_elem(float th0, float* __restrict__ aux, const ModelPack& p, int t, int64_t e,
                                             float beta, float c, float c2) {
  if (KIND == 1) {
    float h = *aux;
    for (int m = 0; m < p.ns; ++m) h = fmaf(c, p.src[m][t][e] - th0, h);
    *aux = h;
    if (!FOLD) return th0;
  }
  float a = th0;
  if (FOLD) {
    a = INIT == 0 ? th0 * beta : th0;
    for (int m = 0; m < p.ns; ++m) a = fmaf(p.w[m], p.src[m][t][e], a);
  }
  if (KIND == 2) return fmaf(c2, FOLD ? th0 : *aux, a * c);
  return a;
}

template <int KIND, bool FOLD, int INIT>
__global__ __launch_bounds__(kThreads) void server_fold_kernel(ModelPack p, float beta, float c, float c2) {
  const int b = blockIdx.x;
  const int t = pack_entry<kModelT>(p.blk0, p.nt, b);  // (uniform)
  float* __restrict__ dst = p.dst[t];
  float* __restrict__ aux = p.theta[t];
  const int64_t n = p.n[t];
  const int64_t c0 = (int64_t)(b - p.blk0[t]) * kModelChunk;
  const int64_t c1 = c0 + kModelChunk < n ? c0 + kModelChunk : n;
  if ((p.vec >> t) & 1u) {
    for (int64_t i = c0 + 4 * (int64_t)threadIdx.x; i < c1; i += 4 * kThreads) {
      if (i + 4 > c1) {  // the tensor's n % 4 tail
        for (int64_t e = i; e < c1; ++e) dst[e] = server_elem<KIND, FOLD, INIT>(dst[e], aux + e, p, t, e, beta, c, c2);
        break;
      }
      // every operand's float4 loaded first, then the chains in message order (weighted_sum's shape)
      float4 sv[kMaxSrc];
#pragma unroll
      for (int m = 0; m < kMaxSrc; ++m)
        if (m < p.ns) sv[m] = *reinterpret_cast<const float4*>(p.src[m][t] + i);
      const float4 t0 = *reinterpret_cast<const float4*>(dst + i);
      // FedDyn: h; pFedMe !FOLD: the saved θ0.  pFedMe's FOLD form never reads aux (its caller passes θ itself there,
      // which the __restrict__ qualifiers would make undefined to load)
      float4 x = (KIND == 1 || !FOLD) ? *reinterpret_cast<const float4*>(aux + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 a = t0;
      if (KIND == 1) {
#pragma unroll
        for (int m = 0; m < kMaxSrc; ++m)
          if (m < p.ns)
            x = make_float4(fmaf(c, sv[m].x - t0.x, x.x), fmaf(c, sv[m].y - t0.y, x.y), fmaf(c, sv[m].z - t0.z, x.z),
                            fmaf(c, sv[m].w - t0.w, x.w));
        *reinterpret_cast<float4*>(aux + i) = x;
      }
      if (FOLD) {
        if (INIT == 0) a = make_float4(t0.x * beta, t0.y * beta, t0.z * beta, t0.w * beta);
#pragma unroll
        for (int m = 0; m < kMaxSrc; ++m) {
          if (m < p.ns) {
            const float w = p.w[m];
            a = make_float4(fmaf(w, sv[m].x, a.x), fmaf(w, sv[m].y, a.y), fmaf(w, sv[m].z, a.z), fmaf(w, sv[m].w, a.w));
          }
        }
      }
      if (KIND == 2) {
        const float4 pr = FOLD ? t0 : x;
        a = make_float4(fmaf(c2, pr.x, a.x * c), fmaf(c2, pr.y, a.y * c), fmaf(c2, pr.z, a.z * c),
                        fmaf(c2, pr.w, a.w * c));
      }
      if (KIND == 2 || FOLD) *reinterpret_cast<float4*>(dst + i) = a;
    }
    return;
  }
  for (int64_t e = c0 + threadIdx.x; e < c1; e += kThreads)
    dst[e] = server_elem<KIND, FOLD, INIT>(dst[e], aux + e, p, t, e, beta, c, c2);
}

// up to 64 blocks of 256 threads per CU of a 256-CU device, grid-stride beyond (tools/wsum_probe.hip, 8 x 25 M:
// 16 K blocks 160-162 us against 169-170 us for 4 K, 163 us for one float4 per thread; profiles/r03/r03p_wsum2.txt)
unsigned grid_for(int64_t work) {
  const int64_t g = cdiv(work, kThreads);
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 64));
}

}  // namespace
}  // namespace flc

using namespace flc;

extern "C" {

int flc_weighted_sum(const float* const* srcs, const float* weights, int n_src, int64_t n, int init_mode, float beta,
                     float* dst, void* stream) {
  if (!dst || n < 0 || n_src < 0 || (n_src > 0 && (!srcs || !weights)))
    return fail(FLC_EINVAL, "flc_weighted_sum: bad arguments");
  if (init_mode < 0 || init_mode > 2) return fail(FLC_EINVAL, "flc_weighted_sum: init_mode must be 0, 1 or 2");
  if (n == 0) return FLC_OK;
  hipStream_t st = as_stream(stream);
  bool vec = (n % 4 == 0) && aligned16(dst);
  for (int m = 0; m < n_src; ++m) {
    if (!srcs[m]) return fail(FLC_EINVAL, "flc_weighted_sum: null source %d", m);
    vec = vec && aligned16(srcs[m]);
  }
  int done = 0;
  int mode = init_mode;
  do {
    SrcPack p;
    p.n = std::min(kMaxSrc, n_src - done);
    for (int m = 0; m < p.n; ++m) {
      p.p[m] = srcs[done + m];
      p.w[m] = weights[done + m];
    }
    for (int m = p.n; m < kMaxSrc; ++m) {
      p.p[m] = nullptr;
      p.w[m] = 0.f;
    }
    const unsigned grid = grid_for(vec ? n / 4 : n);
#define FLC_WS(I, V) FLC_LAUNCH("weighted_sum", (weighted_sum_kernel<I, V>), dim3(grid), dim3(kThreads), 0, st, p, n, beta, dst)
    if (mode == 0) { if (vec) FLC_WS(0, true); else FLC_WS(0, false); }
    else if (mode == 1) { if (vec) FLC_WS(1, true); else FLC_WS(1, false); }
    else { if (vec) FLC_WS(2, true); else FLC_WS(2, false); }
#undef FLC_WS
    done += p.n;
    mode = 2;  // later chunks continue the same fmaf chain
  } while (done < n_src);
  return FLC_OK;
}

int flc_model_fold(float* const* dst, const float* const* srcs, const float* weights, int n_src, const int64_t* sizes,
                   int n_tensors, int init_mode, float beta, float* const* theta, float* const* v, int opt, double lr,
                   double beta2, double tau, void* stream) {
  if (n_tensors < 0 || (n_tensors > 0 && (!dst || !sizes)) || n_src < 0 || n_src > kMaxSrc ||
      (n_src > 0 && (!srcs || !weights)))
    return fail(FLC_EINVAL, "flc_model_fold: bad arguments (at most %d sources)", kMaxSrc);
  if (init_mode < 0 || init_mode > 2) return fail(FLC_EINVAL, "flc_model_fold: init_mode must be 0, 1 or 2");
  const bool step = theta != nullptr;
  if (step && opt != FLC_OPT_AVG && opt != FLC_OPT_ADAGRAD && opt != FLC_OPT_YOGI && opt != FLC_OPT_ADAM)
    return fail(FLC_EINVAL, "flc_model_fold: unknown optimiser %d", opt);
  if (step && opt != FLC_OPT_AVG && !v) return fail(FLC_EINVAL, "flc_model_fold: v required for adaptive optimisers");
  hipStream_t st = as_stream(stream);
  const float omb = (float)(1.0 - beta2), nomb = (float)(-(1.0 - beta2));
  const float lrf = (float)lr, b2f = (float)beta2, tauf = (float)tau;
  for (int t0 = 0; t0 < n_tensors; t0 += kModelT) {
    ModelPack p{};
    p.ns = n_src;
    for (int m = 0; m < n_src; ++m) p.w[m] = weights[m];
    int blocks = 0;
    for (int t = t0; t < std::min(n_tensors, t0 + kModelT); ++t) {
      if (sizes[t] < 0) return fail(FLC_EINVAL, "flc_model_fold: negative size for tensor %d", t);
      if (sizes[t] == 0) continue;
      if (!dst[t] || (step && !theta[t]) || (step && opt != FLC_OPT_AVG && !v[t]))
        return fail(FLC_EINVAL, "flc_model_fold: null pointer for tensor %d", t);
      const int i = p.nt++;
      p.dst[i] = dst[t];
      p.theta[i] = step ? theta[t] : nullptr;
      p.v[i] = (step && v) ? v[t] : nullptr;
      p.n[i] = sizes[t];
      bool vec = aligned16(dst[t]) && (!step || aligned16(theta[t])) && (!p.v[i] || aligned16(p.v[i]));
      for (int m = 0; m < n_src; ++m) {
        const float* sp = srcs[(size_t)m * n_tensors + t];
        if (!sp) return fail(FLC_EINVAL, "flc_model_fold: null source %d of tensor %d", m, t);
        p.src[m][i] = sp;
        vec = vec && aligned16(sp);
      }
      if (vec) p.vec |= 1u << i;
      p.blk0[i] = blocks;
      const int64_t nb = cdiv(sizes[t], kModelChunk);
      if (blocks + nb > 0x7fffffff) return fail(FLC_EINVAL, "flc_model_fold: too many elements");
      blocks += (int)nb;
    }
    p.blk0[p.nt] = blocks;
    if (blocks == 0) continue;
#define FLC_MF(I, O) FLC_LAUNCH("model_fold", (model_fold_kernel<I, O>), dim3(blocks), dim3(kThreads), 0, st, p, beta, lrf, b2f, omb, nomb, tauf)
#define FLC_MF_OPT(I)                                          \
    if (!step) FLC_MF(I, -1);                                   \
    else if (opt == FLC_OPT_AVG) FLC_MF(I, FLC_OPT_AVG);        \
    else if (opt == FLC_OPT_ADAGRAD) FLC_MF(I, FLC_OPT_ADAGRAD); \
    else if (opt == FLC_OPT_YOGI) FLC_MF(I, FLC_OPT_YOGI);      \
    else FLC_MF(I, FLC_OPT_ADAM)
    if (init_mode == 0) { FLC_MF_OPT(0); }
    else if (init_mode == 1) { FLC_MF_OPT(1); }
    else { FLC_MF_OPT(2); }
#undef FLC_MF_OPT
#undef FLC_MF
  }
  return FLC_OK;
}

int flc_avg_and_gradients(float* const* params, float* const* grads, const float* const* param_srcs,
                          const float* const* grad_srcs, const float* w_params, const float* w_grads, int n_src,
                          const int64_t* sizes, int n_tensors, float inertia, void* stream) {
  if (n_tensors < 0 || (n_tensors > 0 && (!params || !grads || !sizes)) || n_src < 1 ||
      !param_srcs || !grad_srcs || !w_params || !w_grads)
    return fail(FLC_EINVAL, "flc_avg_and_gradients: bad arguments");
  hipStream_t st = as_stream(stream);
  for (int t = 0; t < n_tensors; ++t) {
    if (sizes[t] < 0) return fail(FLC_EINVAL, "flc_avg_and_gradients: negative size for tensor %d", t);
    if (sizes[t] > 0 && (!params[t] || !grads[t]))
      return fail(FLC_EINVAL, "flc_avg_and_gradients: null pointer for tensor %d", t);
    for (int m = 0; m < n_src; ++m)
      if (sizes[t] > 0 && (!param_srcs[(size_t)m * n_tensors + t] || !grad_srcs[(size_t)m * n_tensors + t]))
        return fail(FLC_EINVAL, "flc_avg_and_gradients: null source %d of tensor %d", m, t);
  }
  // entries: parameter t, then gradient t, for every non-empty tensor; packed kModelT per launch; messages
  // kMaxSrc per launch (a later chunk continues each chain from the stored partial result: init 2)
  for (int m0 = 0; m0 < n_src; m0 += kMaxSrc) {
    const int ns = std::min(kMaxSrc, n_src - m0);
    int e = 0;  // entry index over 2 * n_tensors
    while (e < 2 * n_tensors) {
      PairPack p{};
      p.ns = ns;
      for (int m = 0; m < ns; ++m) {
        p.w[m] = w_params[m0 + m];
        p.w2[m] = w_grads[m0 + m];
      }
      int blocks = 0;
      for (; e < 2 * n_tensors && p.nt < kModelT; ++e) {
        const int t = e >> 1;
        const bool g = e & 1;
        if (sizes[t] == 0) continue;
        const int i = p.nt++;
        p.dst[i] = g ? grads[t] : params[t];
        p.n[i] = sizes[t];
        p.init[i] = m0 > 0 ? 2 : (g ? 1 : 0);
        if (g) p.grad |= 1u << i;
        bool vec = aligned16(p.dst[i]);
        for (int m = 0; m < ns; ++m) {
          const float* sp = (g ? grad_srcs : param_srcs)[(size_t)(m0 + m) * n_tensors + t];
          p.src[m][i] = sp;
          vec = vec && aligned16(sp);
        }
        if (vec) p.vec |= 1u << i;
        p.blk0[i] = blocks;
        const int64_t nb = cdiv(sizes[t], kModelChunk);
        if (blocks + nb > 0x7fffffff) return fail(FLC_EINVAL, "flc_avg_and_gradients: too many elements");
        blocks += (int)nb;
      }
      p.blk0[p.nt] = blocks;
      if (blocks > 0)
        FLC_LAUNCH("avg_and_gradients", pair_fold_kernel, dim3(blocks), dim3(kThreads), 0, st, p, inertia);
    }
  }
  return FLC_OK;
}

int flc_model_fold_server(float* const* theta, float* const* aux, const float* const* srcs, const float* weights,
                          int n_src, const int64_t* sizes, int n_tensors, int kind, int fold, int init_mode,
                          float inertia, double c, void* stream) {
  if (n_tensors < 0 || (n_tensors > 0 && (!theta || !aux || !sizes)) || n_src < 0 || n_src > kMaxSrc ||
      (n_src > 0 && (!srcs || !weights)))
    return fail(FLC_EINVAL, "flc_model_fold_server: bad arguments (at most %d sources)", kMaxSrc);
  if (kind != FLC_SRV_FEDDYN && kind != FLC_SRV_PFEDME) return fail(FLC_EINVAL, "flc_model_fold_server: unknown kind %d", kind);
  if (init_mode != 0 && init_mode != 2) return fail(FLC_EINVAL, "flc_model_fold_server: init_mode must be 0 or 2");
  if (kind == FLC_SRV_PFEDME && !fold && n_src != 0)
    return fail(FLC_EINVAL, "flc_model_fold_server: the pFedMe blend alone takes no sources");
  hipStream_t st = as_stream(stream);
  // the reference's scalars are Python doubles cast to fp32 by torch: FedDyn alpha = -mu/N, pFedMe beta and 1 - beta
  const float cf = (float)c, c2f = (float)(1.0 - c);
  for (int t0 = 0; t0 < n_tensors; t0 += kModelT) {
    ModelPack p{};
    p.ns = n_src;
    for (int m = 0; m < n_src; ++m) p.w[m] = weights[m];
    int blocks = 0;
    for (int t = t0; t < std::min(n_tensors, t0 + kModelT); ++t) {
      if (sizes[t] < 0) return fail(FLC_EINVAL, "flc_model_fold_server: negative size for tensor %d", t);
      if (sizes[t] == 0) continue;
      if (!theta[t] || !aux[t]) return fail(FLC_EINVAL, "flc_model_fold_server: null pointer for tensor %d", t);
      const int i = p.nt++;
      p.dst[i] = theta[t];
      p.theta[i] = aux[t];
      p.n[i] = sizes[t];
      bool vec = aligned16(theta[t]) && aligned16(aux[t]);
      for (int m = 0; m < n_src; ++m) {
        const float* sp = srcs[(size_t)m * n_tensors + t];
        if (!sp) return fail(FLC_EINVAL, "flc_model_fold_server: null source %d of tensor %d", m, t);
        p.src[m][i] = sp;
        vec = vec && aligned16(sp);
      }
      if (vec) p.vec |= 1u << i;
      p.blk0[i] = blocks;
      const int64_t nb = cdiv(sizes[t], kModelChunk);
      if (blocks + nb > 0x7fffffff) return fail(FLC_EINVAL, "flc_model_fold_server: too many elements");
      blocks += (int)nb;
    }
    p.blk0[p.nt] = blocks;
    if (blocks == 0) continue;
#define FLC_SF(K, F, I) \
  FLC_LAUNCH("model_fold_server", (server_fold_kernel<K, F, I>), dim3(blocks), dim3(kThreads), 0, st, p, inertia, cf, c2f)
    if (kind == FLC_SRV_FEDDYN) {
      if (!fold) FLC_SF(FLC_SRV_FEDDYN, false, 0);
      else if (init_mode == 0) FLC_SF(FLC_SRV_FEDDYN, true, 0);
      else FLC_SF(FLC_SRV_FEDDYN, true, 2);
    } else {
      if (!fold) FLC_SF(FLC_SRV_PFEDME, false, 2);
      else if (init_mode == 0) FLC_SF(FLC_SRV_PFEDME, true, 0);
      else FLC_SF(FLC_SRV_PFEDME, true, 2);
    }
#undef FLC_SF
  }
  return FLC_OK;
}

int flc_fedopt_step(float* theta, const float* delta, float* v, int64_t n, int opt, double lr, double beta2,
                    double tau, void* stream) {
  if (!theta || !delta || n < 0) return fail(FLC_EINVAL, "flc_fedopt_step: bad arguments");
  if (opt != FLC_OPT_AVG && !v) return fail(FLC_EINVAL, "flc_fedopt_step: v required for adaptive optimisers");
  if (n == 0) return FLC_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = grid_for(n);
  // the reference forms 1 - beta2 and -(1 - beta2) as Python doubles; torch casts each scalar to fp32
  const float omb = (float)(1.0 - beta2), nomb = (float)(-(1.0 - beta2));
  const float lrf = (float)lr, b2f = (float)beta2, tauf = (float)tau;
#define FLC_FO(O) FLC_LAUNCH("fedopt_step", fedopt_step_kernel<O>, dim3(grid), dim3(kThreads), 0, st, theta, delta, v, n, lrf, b2f, omb, nomb, tauf)
  switch (opt) {
    case FLC_OPT_AVG: FLC_FO(FLC_OPT_AVG); break;
    case FLC_OPT_ADAGRAD: FLC_FO(FLC_OPT_ADAGRAD); break;
    case FLC_OPT_YOGI: FLC_FO(FLC_OPT_YOGI); break;
    case FLC_OPT_ADAM: FLC_FO(FLC_OPT_ADAM); break;
    default: return fail(FLC_EINVAL, "flc_fedopt_step: unknown optimiser %d", opt);
  }
#undef FLC_FO
  return FLC_OK;
}

int flc_weighted_sum_f64(const double* const* srcs, const double* weights, int n_src, int64_t n, int init_mode,
                         double beta, double* dst, void* stream) {
  if (!dst || n < 0 || n_src < 0 || (n_src > 0 && (!srcs || !weights)))
    return fail(FLC_EINVAL, "flc_weighted_sum_f64: bad arguments");
  if (init_mode < 0 || init_mode > 2) return fail(FLC_EINVAL, "flc_weighted_sum_f64: init_mode must be 0, 1 or 2");
  if (n == 0) return FLC_OK;
  hipStream_t st = as_stream(stream);
  bool vec = (n % 2 == 0) && aligned16(dst);
  for (int m = 0; m < n_src; ++m) {
    if (!srcs[m]) return fail(FLC_EINVAL, "flc_weighted_sum_f64: null source %d", m);
    vec = vec && aligned16(srcs[m]);
  }
  int done = 0, mode = init_mode;
  do {
    SrcPack64 p;
    p.n = std::min(kMaxSrc, n_src - done);
    for (int m = 0; m < kMaxSrc; ++m) {
      p.p[m] = m < p.n ? srcs[done + m] : nullptr;
      p.w[m] = m < p.n ? weights[done + m] : 0.0;
    }
    const unsigned grid = grid_for(vec ? n / 2 : n);
#define FLC_WS(I, V) FLC_LAUNCH("weighted_sum_f64", (weighted_sum64_kernel<I, V>), dim3(grid), dim3(kThreads), 0, st, p, n, beta, dst)
    if (mode == 0) { if (vec) FLC_WS(0, true); else FLC_WS(0, false); }
    else if (mode == 1) { if (vec) FLC_WS(1, true); else FLC_WS(1, false); }
    else { if (vec) FLC_WS(2, true); else FLC_WS(2, false); }
#undef FLC_WS
    done += p.n;
    mode = 2;
  } while (done < n_src);
  return FLC_OK;
}

int flc_fedopt_step_f64(double* theta, const double* delta, double* v, int64_t n, int opt, double lr, double beta2,
                        double tau, void* stream) {
  if (!theta || !delta || n < 0) return fail(FLC_EINVAL, "flc_fedopt_step_f64: bad arguments");
  if (opt != FLC_OPT_AVG && !v) return fail(FLC_EINVAL, "flc_fedopt_step_f64: v required for adaptive optimisers");
  if (n == 0) return FLC_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = grid_for(n);
  const double omb = 1.0 - beta2, nomb = -(1.0 - beta2);  // Python doubles, kept double by float64 torch ops
#define FLC_FO(O) FLC_LAUNCH("fedopt_step_f64", fedopt_step64_kernel<O>, dim3(grid), dim3(kThreads), 0, st, theta, delta, v, n, lr, beta2, omb, nomb, tau)
  switch (opt) {
    case FLC_OPT_AVG: FLC_FO(FLC_OPT_AVG); break;
    case FLC_OPT_ADAGRAD: FLC_FO(FLC_OPT_ADAGRAD); break;
    case FLC_OPT_YOGI: FLC_FO(FLC_OPT_YOGI); break;
    case FLC_OPT_ADAM: FLC_FO(FLC_OPT_ADAM); break;
    default: return fail(FLC_EINVAL, "flc_fedopt_step_f64: unknown optimiser %d", opt);
  }
#undef FLC_FO
  return FLC_OK;
}

int flc_feddr_combine_f64(double* theta, double* y, const double* x_til, int64_t n, double alpha, double cx, double cy,
                          int prox, double prox_c, void* stream) {
  if (!theta || !y || !x_til || n < 0) return fail(FLC_EINVAL, "flc_feddr_combine_f64: bad arguments");
  if (n == 0) return FLC_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = grid_for(n);
#define FLC_DR(P) FLC_LAUNCH("feddr_combine_f64", feddr_combine64_kernel<P>, dim3(grid), dim3(kThreads), 0, st, theta, y, x_til, n, alpha, cx, cy, prox_c)
  switch (prox) {
    case FLC_PROX_NONE: FLC_DR(FLC_PROX_NONE); break;
    case FLC_PROX_L1: FLC_DR(FLC_PROX_L1); break;
    case FLC_PROX_SCALE: FLC_DR(FLC_PROX_SCALE); break;
    default: return fail(FLC_EINVAL, "flc_feddr_combine_f64: unknown prox %d", prox);
  }
#undef FLC_DR
  return FLC_OK;
}

int flc_feddr_combine(float* theta, float* y, const float* x_til, int64_t n, float alpha, float cx, float cy,
                      int prox, float prox_c, void* stream) {
  if (!theta || !y || !x_til || n < 0) return fail(FLC_EINVAL, "flc_feddr_combine: bad arguments");
  if (n == 0) return FLC_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = grid_for(n);
#define FLC_DR(P) FLC_LAUNCH("feddr_combine", feddr_combine_kernel<P>, dim3(grid), dim3(kThreads), 0, st, theta, y, x_til, n, alpha, cx, cy, prox_c)
  switch (prox) {
    case FLC_PROX_NONE: FLC_DR(FLC_PROX_NONE); break;
    case FLC_PROX_L1: FLC_DR(FLC_PROX_L1); break;
    case FLC_PROX_SCALE: FLC_DR(FLC_PROX_SCALE); break;
    default: return fail(FLC_EINVAL, "flc_feddr_combine: unknown prox %d", prox);
  }
#undef FLC_DR
  return FLC_OK;
}

}  // extern "C"

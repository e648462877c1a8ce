// torch_ops.cpp — `torch.ops.flcodec.*`: the codec and aggregation entry points of include/flcodec.h registered
// with the PyTorch dispatcher, so that graph code, torch.compile and other C++ callers
// reach the gfx950 kernels without the ctypes layer.
//
// This is a thin adapter over the same C ABI (libflcodec.so, linked with rpath $ORIGIN): tensors in, tensors out,
// every launch on the current HIP stream of the input's device, nothing synchronised.  The functional ops have
// Meta kernels too (output shapes only), so they trace under FakeTensor.  Each op names the reference lines it
// stands for through the C-ABI function it calls (see the header's comments).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "flcodec.h"

namespace {

constexpr int64_t kTile = FLC_TILE;

void check(int rc, const char* what) {
  TORCH_CHECK(rc == FLC_OK, "flcodec: ", what, " failed with status ", rc, ": ", flc_last_error());
}

void* stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

// fp32, on a HIP device, contiguous and 16-byte aligned (the kernels' vector loads); copies once otherwise
at::Tensor dev_f32(const at::Tensor& x, const char* name) {
  TORCH_CHECK(x.is_cuda(), "flcodec: ", name, " must be on a HIP device (got ", x.device(), ")");
  TORCH_CHECK(x.scalar_type() == at::kFloat, "flcodec: ", name, " must be float32 (got ", x.scalar_type(), ")");
  if (!x.is_contiguous() || reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 != 0) return x.contiguous().clone();
  return x;
}

void same_device(const at::Tensor& a, const at::Tensor& b, const char* name) {
  TORCH_CHECK(b.is_cuda() && b.device() == a.device(), "flcodec: ", name, " must be on ", a.device());
}

// Zero-filled workspace per (device, stream, kind), grown on demand (the C ABI's contract: zero once, then reuse on
// the same stream).  Leaked on purpose: tensors must not be freed after the HIP runtime has gone at exit.
at::Tensor workspace(const at::Tensor& like, size_t nbytes, int kind) {
  static std::mutex mu;
  static auto* cache = new std::map<std::tuple<int, void*, int>, at::Tensor>();
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_tuple((int)like.device().index(), stream_of(like), kind);
  auto it = cache->find(key);
  if (it == cache->end() || (size_t)it->second.numel() < nbytes) {
    at::Tensor t = at::zeros({(int64_t)std::max<size_t>(nbytes, 256)}, like.options().dtype(at::kByte));
    (*cache)[key] = t;
    return t;
  }
  return it->second;
}
enum { kWsQuant = 0, kWsNatural = 1, kWsTopk = 2, kWsAdaptive = 3, kWsTopkBatch = 4 };

int code_bits(int64_t levels) {
  TORCH_CHECK(levels >= 1, "flcodec: levels must be >= 1");
  const int b = 1 + (int)std::ceil(std::log2((double)levels + 1.0));
  for (int c : {2, 4, 8})
    if (b <= c) return c;
  TORCH_CHECK(false, "flcodec: levels=", levels, " does not fit an 8-bit code (at most 127 levels)");
  return 0;
}

int64_t n_tiles(int64_t n) { return (n + kTile - 1) / kTile + 1; }

int norm_kind(int64_t p) {
  TORCH_CHECK(p == 0 || p == 2, "flcodec: p must be 0 (inf norm) or 2");
  return p == 0 ? FLC_NORM_INF : FLC_NORM_L2;
}

// ------------------------------------------------------------------------------------------- stacked codec
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> stacked_encode(const at::Tensor& x_, int64_t k,
                                                                            int64_t levels, int64_t seed,
                                                                            int64_t counter) {
  at::Tensor x = dev_f32(x_, "x").reshape({-1});
  c10::DeviceGuard g(x.device());
  const int64_t n = x.numel();
  at::Tensor idx = at::empty({k}, x.options().dtype(at::kInt));
  at::Tensor codes = at::empty({std::max<int64_t>(k, 16)}, x.options().dtype(at::kByte));
  at::Tensor norm = at::empty({1}, x.options());
  at::Tensor tiles = at::empty({n_tiles(n)}, x.options().dtype(at::kInt));
  at::Tensor ws = workspace(x, flc_topk_workspace_size(n, k), kWsTopk);
  check(flc_stacked_encode_tiled(x.data_ptr<float>(), n, k, (int)levels, (uint64_t)seed, (uint64_t)counter, nullptr,
                                 idx.data_ptr<int32_t>(), codes.data_ptr<uint8_t>(), norm.data_ptr<float>(),
                                 reinterpret_cast<uint32_t*>(tiles.data_ptr<int32_t>()), ws.data_ptr(),
                                 (size_t)ws.numel(), stream_of(x)),
        "stacked_encode");
  return {idx, codes.narrow(0, 0, k), norm, tiles};
}

// packed wire records (flc_stacked_wire_layout): the encode straight into one record, and the one-pass fold of many
// every client's packed wire record from one batched launch (flc_stacked_encode_batch): row c equals
// stacked_encode_wire(xs[c], k, levels, seeds[c], counter)
at::Tensor stacked_encode_batch_wire(at::TensorList xs_, int64_t k, int64_t levels, at::IntArrayRef seeds,
                                     int64_t counter) {
  TORCH_CHECK(!xs_.empty(), "flcodec: stacked_encode_batch_wire needs at least one client");
  TORCH_CHECK(seeds.size() == xs_.size(), "flcodec: one seed per client");
  std::vector<at::Tensor> xs;
  for (const auto& t : xs_) xs.push_back(dev_f32(t, "xs").reshape({-1}));
  c10::DeviceGuard g(xs[0].device());
  const int64_t n = xs[0].numel();
  const int C = (int)xs.size();
  for (const auto& t : xs)
    TORCH_CHECK(t.numel() == n && t.device() == xs[0].device(), "flcodec: clients of one size on one device");
  int64_t off[4];
  const size_t stride = flc_stacked_wire_layout(n, k, off);
  TORCH_CHECK(stride > 0, "flcodec: bad wire shape n=", n, ", k=", k);
  at::Tensor recs = at::empty({(int64_t)C, (int64_t)stride}, xs[0].options().dtype(at::kByte));
  uint8_t* r0 = recs.data_ptr<uint8_t>();
  std::vector<const float*> xp;
  std::vector<uint64_t> sd;
  std::vector<int32_t*> ip;
  std::vector<uint8_t*> cp;
  std::vector<float*> np_;
  std::vector<uint32_t*> tp;
  for (int c = 0; c < C; ++c) {
    uint8_t* r = r0 + (size_t)c * stride;
    xp.push_back(xs[c].data_ptr<float>());
    sd.push_back((uint64_t)seeds[c]);
    ip.push_back(reinterpret_cast<int32_t*>(r + off[1]));
    cp.push_back(r + off[2]);
    np_.push_back(reinterpret_cast<float*>(r + off[0]));
    tp.push_back(reinterpret_cast<uint32_t*>(r + off[3]));
  }
  at::Tensor ws = workspace(xs[0], flc_stacked_encode_batch_workspace_size(n, k, C), kWsTopkBatch);
  check(flc_stacked_encode_batch(xp.data(), C, n, k, (int)levels, sd.data(), (uint64_t)counter, ip.data(), cp.data(),
                                 np_.data(), tp.data(), ws.data_ptr(), (size_t)ws.numel(), stream_of(xs[0])),
        "stacked_encode_batch_wire");
  return recs;
}

at::Tensor stacked_encode_wire(const at::Tensor& x_, int64_t k, int64_t levels, int64_t seed, int64_t counter) {
  at::Tensor x = dev_f32(x_, "x").reshape({-1});
  c10::DeviceGuard g(x.device());
  const int64_t n = x.numel();
  int64_t off[4];
  const size_t stride = flc_stacked_wire_layout(n, k, off);
  TORCH_CHECK(stride > 0, "flcodec: bad wire shape n=", n, ", k=", k);
  at::Tensor rec = at::empty({(int64_t)stride}, x.options().dtype(at::kByte));
  uint8_t* r = rec.data_ptr<uint8_t>();
  at::Tensor ws = workspace(x, flc_topk_workspace_size(n, k), kWsTopk);
  check(flc_stacked_encode_tiled(x.data_ptr<float>(), n, k, (int)levels, (uint64_t)seed, (uint64_t)counter, nullptr,
                                 reinterpret_cast<int32_t*>(r + off[1]), r + off[2], reinterpret_cast<float*>(r + off[0]),
                                 reinterpret_cast<uint32_t*>(r + off[3]), ws.data_ptr(), (size_t)ws.numel(),
                                 stream_of(x)),
        "stacked_encode_wire");
  return rec;
}

at::Tensor stacked_fold_wires(const at::Tensor& wires, at::IntArrayRef slots, at::ArrayRef<double> weights, int64_t n,
                              int64_t k, int64_t levels, const c10::optional<at::Tensor>& out_, bool accumulate) {
  TORCH_CHECK(wires.is_cuda() && wires.scalar_type() == at::kByte && wires.is_contiguous(),
              "flcodec: wires must be a contiguous uint8 HIP tensor");
  TORCH_CHECK(slots.size() == weights.size() && !slots.empty(), "flcodec: one weight per slot, at least one");
  const int64_t stride = wires.dim() == 2 ? wires.size(1) : (int64_t)flc_stacked_wire_layout(n, k, nullptr);
  TORCH_CHECK(stride > 0, "flcodec: bad wire shape n=", n, ", k=", k);
  const int64_t nrec = wires.numel() / stride;
  std::vector<int32_t> sl(slots.size());
  std::vector<float> wt(weights.size());
  for (size_t c = 0; c < slots.size(); ++c) {
    TORCH_CHECK(slots[c] >= 0 && slots[c] < nrec, "flcodec: slot ", slots[c], " outside the ", nrec, " records");
    sl[c] = (int32_t)slots[c];
    wt[c] = (float)weights[c];
  }
  at::Tensor out;
  if (out_.has_value()) {
    out = *out_;
    same_device(out, wires, "wires");
    TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == n,
                "flcodec: out must be a contiguous fp32 tensor of n elements");
  } else {
    TORCH_CHECK(!accumulate, "flcodec: accumulate needs an out tensor");
    out = at::empty({n}, wires.options().dtype(at::kFloat));
  }
  c10::DeviceGuard g(wires.device());
  check(flc_stacked_fold_wires(wires.data_ptr(), stride, sl.data(), wt.data(), (int)sl.size(), n, k, (int)levels,
                               accumulate ? 1 : 0, out.data_ptr<float>(), stream_of(out)),
        "stacked_fold_wires");
  return out;
}

void stacked_decode_into(at::Tensor& out, const at::Tensor& idx, const at::Tensor& codes, const at::Tensor& norm,
                         const at::Tensor& tiles, int64_t levels, double weight, bool accumulate) {
  same_device(out, idx, "idx");
  same_device(out, codes, "codes");
  same_device(out, norm, "norm");
  same_device(out, tiles, "tiles");
  TORCH_CHECK(idx.scalar_type() == at::kInt && codes.scalar_type() == at::kByte && norm.scalar_type() == at::kFloat &&
                  tiles.scalar_type() == at::kInt,
              "flcodec: stacked packet dtypes are (int32 idx, uint8 codes, fp32 norm, int32 tiles)");
  TORCH_CHECK(idx.is_contiguous() && codes.is_contiguous() && tiles.is_contiguous(), "flcodec: packet not contiguous");
  const int64_t n = out.numel(), k = idx.numel();
  TORCH_CHECK(codes.numel() >= k && tiles.numel() == n_tiles(n), "flcodec: packet does not match n=", n, ", k=", k);
  c10::DeviceGuard g(out.device());
  check(flc_stacked_decode_tiled(idx.data_ptr<int32_t>(), codes.data_ptr<uint8_t>(), k, (int)levels,
                                 norm.data_ptr<float>(), n, (float)weight, accumulate ? 1 : 0, out.data_ptr<float>(),
                                 reinterpret_cast<const uint32_t*>(tiles.data_ptr<int32_t>()), stream_of(out)),
        "stacked_decode");
}

at::Tensor stacked_decode(const at::Tensor& idx, const at::Tensor& codes, const at::Tensor& norm,
                          const at::Tensor& tiles, int64_t n, int64_t levels, double weight) {
  at::Tensor out = at::empty({n}, idx.options().dtype(at::kFloat));
  stacked_decode_into(out, idx, codes, norm, tiles, levels, weight, false);
  return out;
}

at::Tensor& stacked_decode_accumulate_(at::Tensor& out, const at::Tensor& idx, const at::Tensor& codes,
                                       const at::Tensor& norm, const at::Tensor& tiles, int64_t levels,
                                       double weight) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous(),
              "flcodec: out must be a contiguous fp32 HIP tensor");
  stacked_decode_into(out, idx, codes, norm, tiles, levels, weight, true);
  return out;
}

// ---------------------------------------------------------------------------------------------------- top-k
std::tuple<at::Tensor, at::Tensor, at::Tensor> topk_encode(const at::Tensor& x_, int64_t k) {
  at::Tensor x = dev_f32(x_, "x").reshape({-1});
  c10::DeviceGuard g(x.device());
  const int64_t n = x.numel();
  at::Tensor idx = at::empty({k}, x.options().dtype(at::kInt));
  at::Tensor val = at::empty({k}, x.options());
  at::Tensor tiles = at::empty({n_tiles(n)}, x.options().dtype(at::kInt));
  at::Tensor ws = workspace(x, flc_topk_workspace_size(n, k), kWsTopk);
  check(flc_topk_encode_tiled(x.data_ptr<float>(), n, k, idx.data_ptr<int32_t>(), val.data_ptr<float>(),
                              reinterpret_cast<uint32_t*>(tiles.data_ptr<int32_t>()), ws.data_ptr(),
                              (size_t)ws.numel(), stream_of(x)),
        "topk_encode");
  return {idx, val, tiles};
}

at::Tensor sparse_decode(const at::Tensor& idx, const at::Tensor& val_, const at::Tensor& tiles, int64_t n,
                         double scale, double weight) {
  at::Tensor val = dev_f32(val_, "val");
  same_device(val, idx, "idx");
  same_device(val, tiles, "tiles");
  TORCH_CHECK(idx.scalar_type() == at::kInt && tiles.scalar_type() == at::kInt && idx.is_contiguous() &&
                  tiles.is_contiguous(),
              "flcodec: idx and tiles must be contiguous int32");
  TORCH_CHECK(idx.numel() == val.numel() && tiles.numel() == n_tiles(n), "flcodec: sparse stream does not match n");
  c10::DeviceGuard g(val.device());
  at::Tensor out = at::empty({n}, val.options());
  check(flc_sparse_decode_tiled(idx.data_ptr<int32_t>(), val.data_ptr<float>(), idx.numel(), (float)scale, n,
                                (float)weight, 0, out.data_ptr<float>(),
                                reinterpret_cast<const uint32_t*>(tiles.data_ptr<int32_t>()), stream_of(out)),
        "sparse_decode");
  return out;
}

// ------------------------------------------------------------------------------------------- dense dithering
at::Tensor quant_norm(const at::Tensor& x_, int64_t p) {
  at::Tensor x = dev_f32(x_, "x");
  TORCH_CHECK(x.dim() == 2, "flcodec: quant_norm takes a [rows, d] batch");
  c10::DeviceGuard g(x.device());
  const int64_t rows = x.size(0), d = x.size(1);
  at::Tensor norms = at::empty({rows}, x.options());
  at::Tensor ws = workspace(x, flc_quant_workspace_size(rows, d), kWsQuant);
  check(flc_quant_norm(x.data_ptr<float>(), rows, d, norm_kind(p), norms.data_ptr<float>(), ws.data_ptr(),
                       (size_t)ws.numel(), stream_of(x)),
        "quant_norm");
  return norms;
}

std::tuple<at::Tensor, at::Tensor> quant_encode(const at::Tensor& x_, const at::Tensor& norms, int64_t kind,
                                                int64_t levels, int64_t seed, int64_t counter) {
  at::Tensor x = dev_f32(x_, "x");
  TORCH_CHECK(x.dim() == 2, "flcodec: quant_encode takes a [rows, d] batch");
  same_device(x, norms, "norms");
  const int64_t rows = x.size(0), d = x.size(1);
  TORCH_CHECK(norms.scalar_type() == at::kFloat && norms.numel() == rows && norms.is_contiguous(),
              "flcodec: norms must be contiguous fp32 of one entry per row");
  c10::DeviceGuard g(x.device());
  const int bits = code_bits(levels);
  at::Tensor codes = at::empty({std::max<int64_t>((rows * d * bits + 7) / 8, 1)}, x.options().dtype(at::kByte));
  at::Tensor nnz = at::empty({rows}, x.options().dtype(at::kLong));
  at::Tensor ws = workspace(x, flc_quant_workspace_size(rows, d), kWsQuant);
  check(flc_quant_encode(x.data_ptr<float>(), rows, d, (int)kind, (int)levels, bits, norms.data_ptr<float>(),
                         (uint64_t)seed, (uint64_t)counter, nullptr, codes.data_ptr<uint8_t>(), nnz.data_ptr<int64_t>(),
                         ws.data_ptr(), (size_t)ws.numel(), stream_of(x)),
        "quant_encode");
  return {codes, nnz};
}

at::Tensor quant_decode(const at::Tensor& codes, const at::Tensor& norms, int64_t d, int64_t kind, int64_t levels) {
  same_device(norms, codes, "codes");
  TORCH_CHECK(codes.scalar_type() == at::kByte && codes.is_contiguous() && norms.scalar_type() == at::kFloat &&
                  norms.is_contiguous(),
              "flcodec: quant packet is (uint8 codes, fp32 norms)");
  const int64_t rows = norms.numel();
  const int bits = code_bits(levels);
  TORCH_CHECK(codes.numel() >= (rows * d * bits + 7) / 8, "flcodec: codes too short for [", rows, ", ", d, "]");
  c10::DeviceGuard g(norms.device());
  at::Tensor out = at::empty({rows, d}, norms.options());
  check(flc_quant_decode(codes.data_ptr<uint8_t>(), rows, d, (int)kind, (int)levels, bits, norms.data_ptr<float>(),
                         nullptr, 0, out.data_ptr<float>(), stream_of(out)),
        "quant_decode");
  return out;
}

// ---------------------------------------------------------------------------------------- natural compressor
std::tuple<at::Tensor, at::Tensor> natural_encode(const at::Tensor& x_, int64_t seed, int64_t counter) {
  at::Tensor x = dev_f32(x_, "x").reshape({-1});
  c10::DeviceGuard g(x.device());
  const int64_t n = x.numel();
  at::Tensor codes = at::empty({n}, x.options().dtype(at::kShort));
  at::Tensor nnz = at::empty({1}, x.options().dtype(at::kLong));
  at::Tensor ws = workspace(x, flc_natural_workspace_size(n), kWsNatural);
  check(flc_natural_encode(x.data_ptr<float>(), n, (uint64_t)seed, (uint64_t)counter, nullptr,
                           reinterpret_cast<uint16_t*>(codes.data_ptr<int16_t>()), nnz.data_ptr<int64_t>(),
                           ws.data_ptr(), (size_t)ws.numel(), stream_of(x)),
        "natural_encode");
  return {codes, nnz};
}

at::Tensor natural_decode(const at::Tensor& codes, double weight) {
  TORCH_CHECK(codes.is_cuda() && codes.scalar_type() == at::kShort && codes.is_contiguous(),
              "flcodec: natural codes must be contiguous int16 on a HIP device");
  c10::DeviceGuard g(codes.device());
  at::Tensor out = at::empty({codes.numel()}, codes.options().dtype(at::kFloat));
  check(flc_natural_decode(reinterpret_cast<const uint16_t*>(codes.data_ptr<int16_t>()), codes.numel(),
                           (float)weight, 0, out.data_ptr<float>(), stream_of(out)),
        "natural_decode");
  return out;
}

// --------------------------------------------------------------------------------------------- aggregation
at::Tensor& weighted_sum_(at::Tensor& dst, at::TensorList srcs, at::ArrayRef<double> weights, int64_t init_mode,
                          double beta) {
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kFloat && dst.is_contiguous(),
              "flcodec: dst must be a contiguous fp32 HIP tensor");
  TORCH_CHECK(srcs.size() == weights.size(), "flcodec: one weight per source");
  TORCH_CHECK(init_mode >= 0 && init_mode <= 2, "flcodec: init_mode is 0 (dst*beta), 1 (zero) or 2 (keep)");
  c10::DeviceGuard g(dst.device());
  std::vector<at::Tensor> keep;
  std::vector<const float*> ptrs;
  std::vector<float> w;
  for (size_t m = 0; m < srcs.size(); ++m) {
    same_device(dst, srcs[m], "every source");
    TORCH_CHECK(srcs[m].numel() == dst.numel(), "flcodec: every source must have dst's number of elements");
    keep.push_back(dev_f32(srcs[m], "src"));
    ptrs.push_back(keep.back().data_ptr<float>());
    w.push_back((float)weights[m]);
  }
  check(flc_weighted_sum(ptrs.data(), w.data(), (int)ptrs.size(), dst.numel(), (int)init_mode, (float)beta,
                         dst.data_ptr<float>(), stream_of(dst)),
        "weighted_sum");
  return dst;
}

// a whole model in one launch (flc_model_fold): dsts[t] per model tensor, srcs[m * n_tensors + t] message-major,
// theta / v empty or one per tensor.  Every tensor is checked here in C++ (device, dtype, contiguity, size): the host
// cost of a model update is these checks plus one launch (a model is ~10-100 small tensors).
void model_fold_(at::TensorList dsts, at::TensorList srcs, at::ArrayRef<double> weights, int64_t init_mode,
                 double beta, at::TensorList theta, at::TensorList v, int64_t opt, double lr, double beta2, double tau) {
  const size_t nt = dsts.size(), ns = weights.size();
  TORCH_CHECK_VALUE(ns <= 16, "flcodec: model_fold takes at most 16 messages");
  TORCH_CHECK_VALUE(srcs.size() == ns * nt, "flcodec: every message has one tensor per model tensor");
  TORCH_CHECK_VALUE(theta.empty() || theta.size() == nt, "flcodec: theta has one tensor per model tensor");
  TORCH_CHECK_VALUE(v.empty() || v.size() == nt, "flcodec: v has one tensor per model tensor");
  if (nt == 0) return;
  const c10::Device dev = dsts[0].device();
  auto usable = [&](const at::Tensor& t) {
    return t.is_cuda() && t.device() == dev && t.scalar_type() == at::kFloat && t.is_contiguous();
  };
  std::vector<float*> dp(nt), tp(theta.size()), vp(v.size());
  std::vector<int64_t> sz(nt);
  for (size_t t = 0; t < nt; ++t) {
    TORCH_CHECK_TYPE(usable(dsts[t]), "flcodec: model tensors must be contiguous fp32 HIP tensors on one device");
    dp[t] = dsts[t].data_ptr<float>();
    sz[t] = dsts[t].numel();
    if (!theta.empty()) {
      TORCH_CHECK_TYPE(usable(theta[t]), "flcodec: theta tensors must be contiguous fp32 HIP tensors on one device");
      TORCH_CHECK_VALUE(theta[t].numel() == sz[t], "flcodec: theta must match the model tensors' sizes");
      tp[t] = theta[t].data_ptr<float>();
    }
    if (!v.empty()) {
      TORCH_CHECK_TYPE(usable(v[t]), "flcodec: v tensors must be contiguous fp32 HIP tensors on one device");
      TORCH_CHECK_VALUE(v[t].numel() == sz[t], "flcodec: v must match the model tensors' sizes");
      vp[t] = v[t].data_ptr<float>();
    }
  }
  std::vector<const float*> sp(ns * nt);
  for (size_t i = 0; i < sp.size(); ++i) {
    const at::Tensor& a = srcs[i];
    TORCH_CHECK_TYPE(usable(a), "flcodec: message tensors must be contiguous fp32 HIP tensors on the model's device");
    TORCH_CHECK_VALUE(a.numel() == sz[i % nt], "flcodec: message tensors must match the model tensors' sizes");
    sp[i] = a.data_ptr<float>();
  }
  std::vector<float> w(ns);
  for (size_t m = 0; m < ns; ++m) w[m] = (float)weights[m];
  c10::DeviceGuard g(dev);
  check(flc_model_fold(dp.data(), sp.data(), w.data(), (int)ns, sz.data(), (int)nt, (int)init_mode, (float)beta,
                       theta.empty() ? nullptr : tp.data(), v.empty() ? nullptr : vp.data(), (int)opt, lr, beta2, tau,
                       stream_of(dsts[0])),
        "model_fold");
}

void fedopt_step_(at::Tensor& theta, const at::Tensor& delta_, const c10::optional<at::Tensor>& v, int64_t opt,
                  double lr, double beta2, double tau) {
  TORCH_CHECK(theta.is_cuda() && theta.scalar_type() == at::kFloat && theta.is_contiguous(),
              "flcodec: theta must be a contiguous fp32 HIP tensor");
  at::Tensor delta = dev_f32(delta_, "delta");
  same_device(theta, delta, "delta");
  TORCH_CHECK(delta.numel() == theta.numel(), "flcodec: delta must match theta");
  TORCH_CHECK(opt >= FLC_OPT_AVG && opt <= FLC_OPT_ADAM, "flcodec: opt is 0 avg, 1 adagrad, 2 yogi, 3 adam");
  float* vp = nullptr;
  if (opt != FLC_OPT_AVG) {
    TORCH_CHECK(v.has_value(), "flcodec: adaptive optimisers need the second-moment tensor v");
    same_device(theta, *v, "v");
    TORCH_CHECK(v->scalar_type() == at::kFloat && v->is_contiguous() && v->numel() == theta.numel(),
                "flcodec: v must be contiguous fp32 like theta");
    vp = v->data_ptr<float>();
  }
  c10::DeviceGuard g(theta.device());
  check(flc_fedopt_step(theta.data_ptr<float>(), delta.data_ptr<float>(), vp, theta.numel(), (int)opt, lr, beta2, tau,
                        stream_of(theta)),
        "fedopt_step");
}

// ------------------------------------------------------------------------------------------- client delta (f1)
at::Tensor delta_flatten(at::TensorList local, at::TensorList global) {
  TORCH_CHECK(local.size() == global.size() && !local.empty(), "flcodec: one global tensor per local tensor");
  std::vector<at::Tensor> keep;
  std::vector<const float*> lp, gp;
  std::vector<int64_t> sz;
  int64_t total = 0;
  for (size_t t = 0; t < local.size(); ++t) {
    same_device(local[0], local[t], "every local tensor");
    same_device(local[0], global[t], "every global tensor");
    TORCH_CHECK(local[t].numel() == global[t].numel(), "flcodec: local and global tensor ", t, " differ in size");
    keep.push_back(dev_f32(local[t], "local"));
    lp.push_back(keep.back().data_ptr<float>());
    keep.push_back(dev_f32(global[t], "global"));
    gp.push_back(keep.back().data_ptr<float>());
    sz.push_back(local[t].numel());
    total += local[t].numel();
  }
  c10::DeviceGuard g(local[0].device());
  at::Tensor out = at::empty({total}, local[0].options());
  check(flc_delta_flatten(lp.data(), gp.data(), sz.data(), (int)sz.size(), total ? out.data_ptr<float>() : nullptr,
                          stream_of(out)),
        "delta_flatten");
  return out;
}

void feddr_combine_(at::Tensor& theta, at::Tensor& y, const at::Tensor& x_til, double alpha, double cx, double cy,
                    int64_t prox, double prox_c) {
  const at::Tensor* all[3] = {&theta, &y, &x_til};
  for (const at::Tensor* t : all) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == theta.numel(),
                "flcodec: theta, y and x_til must be contiguous fp32 HIP tensors of one size");
    same_device(theta, *t, "theta, y and x_til");
  }
  c10::DeviceGuard g(theta.device());
  check(flc_feddr_combine(theta.data_ptr<float>(), y.data_ptr<float>(), x_til.data_ptr<float>(), theta.numel(),
                          (float)alpha, (float)cx, (float)cy, (int)prox, (float)prox_c, stream_of(theta)),
        "feddr_combine");
}

// ------------------------------------------------------------------------------------- round-2 entry points
// the stacked encode of the client delta formed in the encoder's read (flc_stacked_encode_delta)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> stacked_encode_delta(at::TensorList local,
                                                                                  at::TensorList global, int64_t k,
                                                                                  int64_t levels, int64_t seed,
                                                                                  int64_t counter) {
  TORCH_CHECK(!local.empty() && local.size() == global.size(), "flcodec: one global tensor per local tensor");
  std::vector<at::Tensor> keep;
  std::vector<const float*> lp, gp;
  std::vector<int64_t> sz;
  int64_t n = 0;
  for (size_t t = 0; t < local.size(); ++t) {
    same_device(local[0], local[t], "local tensors");
    same_device(local[0], global[t], "global tensors");
    TORCH_CHECK(local[t].numel() == global[t].numel(), "flcodec: local and global tensor ", t, " differ in size");
    keep.push_back(dev_f32(local[t], "local"));
    lp.push_back(keep.back().data_ptr<float>());
    keep.push_back(dev_f32(global[t], "global"));
    gp.push_back(keep.back().data_ptr<float>());
    sz.push_back(local[t].numel());
    n += local[t].numel();
  }
  const at::Tensor& x = local[0];
  c10::DeviceGuard g(x.device());
  at::Tensor idx = at::empty({k}, x.options().dtype(at::kInt));
  at::Tensor codes = at::empty({std::max<int64_t>(k, 16)}, x.options().dtype(at::kByte));
  at::Tensor norm = at::empty({1}, x.options().dtype(at::kFloat));
  at::Tensor tiles = at::empty({n_tiles(n)}, x.options().dtype(at::kInt));
  at::Tensor ws = workspace(x, flc_stacked_encode_delta_workspace_size(n, k, (int)sz.size()), kWsTopk);
  check(flc_stacked_encode_delta(lp.data(), gp.data(), sz.data(), (int)sz.size(), k, (int)levels, (uint64_t)seed,
                                 (uint64_t)counter, idx.data_ptr<int32_t>(), codes.data_ptr<uint8_t>(),
                                 norm.data_ptr<float>(), reinterpret_cast<uint32_t*>(tiles.data_ptr<int32_t>()),
                                 ws.data_ptr(), (size_t)ws.numel(), stream_of(x)),
        "stacked_encode_delta");
  return {idx, codes.narrow(0, 0, k), norm, tiles};
}

// philox dithering with the norm included and the decode fused (flc_quant_encode_auto)
std::tuple<at::Tensor, at::Tensor, at::Tensor> quant_encode_auto(const at::Tensor& x_, int64_t kind, int64_t levels,
                                                                 int64_t p, int64_t seed, int64_t counter) {
  at::Tensor x = dev_f32(x_, "x");
  TORCH_CHECK(x.dim() == 2, "flcodec: quant_encode_auto takes a [rows, d] batch");
  c10::DeviceGuard g(x.device());
  const int64_t rows = x.size(0), d = x.size(1);
  const int bits = code_bits(levels);
  at::Tensor codes = at::empty({std::max<int64_t>((rows * d * bits + 7) / 8, 1)}, x.options().dtype(at::kByte));
  at::Tensor norms = at::empty({rows}, x.options());
  at::Tensor out = at::empty({rows, d}, x.options());
  at::Tensor ws = workspace(x, flc_quant_workspace_size(rows, d), kWsQuant);
  check(flc_quant_encode_auto(x.data_ptr<float>(), rows, d, (int)kind, (int)levels, bits, norm_kind(p), (uint64_t)seed,
                              (uint64_t)counter, codes.data_ptr<uint8_t>(), norms.data_ptr<float>(), nullptr,
                              out.data_ptr<float>(), ws.data_ptr(), (size_t)ws.numel(), stream_of(x)),
        "quant_encode_auto");
  return {codes, norms, out};
}

// adaptive random with the uniform given (flc_adaptive_prepare + flc_adaptive_select): (out, index, status);
// status != 0 is numpy's ValueError (1: p contains NaN, 2: p does not sum to 1) and then out is all zero
std::tuple<at::Tensor, at::Tensor, at::Tensor> adaptive_random(const at::Tensor& x_, double u) {
  at::Tensor x = dev_f32(x_, "x").reshape({-1});
  c10::DeviceGuard g(x.device());
  const int64_t n = x.numel();
  TORCH_CHECK(n > 0, "flcodec: adaptive_random of an empty vector");
  at::Tensor status = at::empty({1}, x.options().dtype(at::kInt));
  at::Tensor index = at::zeros({1}, x.options().dtype(at::kLong));
  at::Tensor out = at::empty({n}, x.options());
  at::Tensor ws = workspace(x, flc_adaptive_workspace_size(n), kWsAdaptive);
  check(flc_adaptive_prepare(x.data_ptr<float>(), n, status.data_ptr<int32_t>(), ws.data_ptr(), (size_t)ws.numel(),
                             stream_of(x)),
        "adaptive_prepare");
  check(flc_adaptive_select(x.data_ptr<float>(), n, u, index.data_ptr<int64_t>(), out.data_ptr<float>(), ws.data_ptr(),
                            (size_t)ws.numel(), stream_of(x)),
        "adaptive_select");
  return {out, index, status};
}

// --------------------------------------------------------------------------------- Meta kernels (shapes only)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> stacked_encode_delta_meta(at::TensorList local,
                                                                                       at::TensorList, int64_t k,
                                                                                       int64_t, int64_t, int64_t) {
  int64_t n = 0;
  for (const auto& t : local) n += t.numel();
  const auto o = local[0].options();
  return {at::empty({k}, o.dtype(at::kInt)), at::empty({k}, o.dtype(at::kByte)), at::empty({1}, o.dtype(at::kFloat)),
          at::empty({n_tiles(n)}, o.dtype(at::kInt))};
}
std::tuple<at::Tensor, at::Tensor, at::Tensor> quant_encode_auto_meta(const at::Tensor& x, int64_t, int64_t levels,
                                                                      int64_t, int64_t, int64_t) {
  const int64_t rows = x.size(0), d = x.size(1);
  return {at::empty({std::max<int64_t>((rows * d * code_bits(levels) + 7) / 8, 1)}, x.options().dtype(at::kByte)),
          at::empty({rows}, x.options()), at::empty({rows, d}, x.options())};
}
std::tuple<at::Tensor, at::Tensor, at::Tensor> adaptive_random_meta(const at::Tensor& x, double) {
  return {at::empty({x.numel()}, x.options()), at::empty({1}, x.options().dtype(at::kLong)),
          at::empty({1}, x.options().dtype(at::kInt))};
}
at::Tensor delta_flatten_meta(at::TensorList local, at::TensorList) {
  int64_t total = 0;
  for (const auto& t : local) total += t.numel();
  return at::empty({total}, local[0].options());
}
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> stacked_encode_meta(const at::Tensor& x, int64_t k,
                                                                                 int64_t, int64_t, int64_t) {
  const int64_t n = x.numel();
  return {at::empty({k}, x.options().dtype(at::kInt)), at::empty({k}, x.options().dtype(at::kByte)),
          at::empty({1}, x.options().dtype(at::kFloat)), at::empty({n_tiles(n)}, x.options().dtype(at::kInt))};
}
at::Tensor stacked_encode_batch_wire_meta(at::TensorList xs, int64_t k, int64_t, at::IntArrayRef, int64_t) {
  TORCH_CHECK(!xs.empty(), "flcodec: stacked_encode_batch_wire needs at least one client");
  return at::empty({(int64_t)xs.size(), (int64_t)flc_stacked_wire_layout(xs[0].numel(), k, nullptr)},
                   xs[0].options().dtype(at::kByte));
}
at::Tensor stacked_encode_wire_meta(const at::Tensor& x, int64_t k, int64_t, int64_t, int64_t) {
  return at::empty({(int64_t)flc_stacked_wire_layout(x.numel(), k, nullptr)}, x.options().dtype(at::kByte));
}
at::Tensor stacked_fold_wires_meta(const at::Tensor& wires, at::IntArrayRef, at::ArrayRef<double>, int64_t n, int64_t,
                                   int64_t, const c10::optional<at::Tensor>&, bool) {
  return at::empty({n}, wires.options().dtype(at::kFloat));
}
at::Tensor stacked_decode_meta(const at::Tensor& idx, const at::Tensor&, const at::Tensor&, const at::Tensor&,
                               int64_t n, int64_t, double) {
  return at::empty({n}, idx.options().dtype(at::kFloat));
}
std::tuple<at::Tensor, at::Tensor, at::Tensor> topk_encode_meta(const at::Tensor& x, int64_t k) {
  return {at::empty({k}, x.options().dtype(at::kInt)), at::empty({k}, x.options().dtype(at::kFloat)),
          at::empty({n_tiles(x.numel())}, x.options().dtype(at::kInt))};
}
at::Tensor sparse_decode_meta(const at::Tensor&, const at::Tensor& val, const at::Tensor&, int64_t n, double, double) {
  return at::empty({n}, val.options().dtype(at::kFloat));
}
at::Tensor quant_norm_meta(const at::Tensor& x, int64_t) { return at::empty({x.size(0)}, x.options()); }
std::tuple<at::Tensor, at::Tensor> quant_encode_meta(const at::Tensor& x, const at::Tensor&, int64_t,
                                                     int64_t levels, int64_t, int64_t) {
  const int64_t rows = x.size(0), d = x.size(1);
  return {at::empty({std::max<int64_t>((rows * d * code_bits(levels) + 7) / 8, 1)}, x.options().dtype(at::kByte)),
          at::empty({rows}, x.options().dtype(at::kLong))};
}
at::Tensor quant_decode_meta(const at::Tensor&, const at::Tensor& norms, int64_t d, int64_t, int64_t) {
  return at::empty({norms.numel(), d}, norms.options());
}
std::tuple<at::Tensor, at::Tensor> natural_encode_meta(const at::Tensor& x, int64_t, int64_t) {
  return {at::empty({x.numel()}, x.options().dtype(at::kShort)), at::empty({1}, x.options().dtype(at::kLong))};
}
at::Tensor natural_decode_meta(const at::Tensor& codes, double) {
  return at::empty({codes.numel()}, codes.options().dtype(at::kFloat));
}

}  // namespace

TORCH_LIBRARY(flcodec, m) {
  m.def("stacked_encode(Tensor x, int k, int levels=127, int seed=0, int counter=0) "
        "-> (Tensor idx, Tensor codes, Tensor norm, Tensor tiles)");
  m.def("stacked_decode(Tensor idx, Tensor codes, Tensor norm, Tensor tiles, int n, int levels=127, "
        "float weight=1.0) -> Tensor");
  m.def("stacked_decode_accumulate_(Tensor(a!) out, Tensor idx, Tensor codes, Tensor norm, Tensor tiles, "
        "int levels=127, float weight=1.0) -> Tensor(a!)");
  m.def("topk_encode(Tensor x, int k) -> (Tensor idx, Tensor val, Tensor tiles)");
  m.def("sparse_decode(Tensor idx, Tensor val, Tensor tiles, int n, float scale=1.0, float weight=1.0) -> Tensor");
  m.def("quant_norm(Tensor x, int p=0) -> Tensor");
  m.def("quant_encode(Tensor x, Tensor norms, int kind, int levels, int seed=0, int counter=0) "
        "-> (Tensor codes, Tensor nnz)");
  m.def("quant_decode(Tensor codes, Tensor norms, int d, int kind, int levels) -> Tensor");
  m.def("natural_encode(Tensor x, int seed=0, int counter=0) -> (Tensor codes, Tensor nnz)");
  m.def("natural_decode(Tensor codes, float weight=1.0) -> Tensor");
  m.def("weighted_sum_(Tensor(a!) dst, Tensor[] srcs, float[] weights, int init_mode, float beta=0.0) -> Tensor(a!)");
  m.def("fedopt_step_(Tensor(a!) theta, Tensor delta, Tensor(b!)? v, int opt, float lr, float beta2, float tau) -> ()");
  m.def("model_fold_(Tensor(a!)[] dsts, Tensor[] srcs, float[] weights, int init_mode, float beta, "
        "Tensor(b!)[] theta, Tensor(c!)[] v, int opt=0, float lr=1.0, float beta2=0.0, float tau=0.0) -> ()");
  m.def("delta_flatten(Tensor[] theta_local, Tensor[] theta_global) -> Tensor");
  m.def("feddr_combine_(Tensor(a!) theta, Tensor(b!) y, Tensor x_til, float alpha, float cx, float cy, int prox, "
        "float prox_c) -> ()");
  m.def("stacked_encode_delta(Tensor[] theta_local, Tensor[] theta_global, int k, int levels=127, int seed=0, "
        "int counter=0) -> (Tensor idx, Tensor codes, Tensor norm, Tensor tiles)");
  m.def("quant_encode_auto(Tensor x, int kind, int levels, int p=0, int seed=0, int counter=0) "
        "-> (Tensor codes, Tensor norms, Tensor decoded)");
  m.def("adaptive_random(Tensor x, float u) -> (Tensor out, Tensor index, Tensor status)");
  m.def("stacked_encode_wire(Tensor x, int k, int levels=127, int seed=0, int counter=0) -> Tensor");
  m.def("stacked_encode_batch_wire(Tensor[] xs, int k, int levels, int[] seeds, int counter=0) -> Tensor");
  m.def("stacked_fold_wires(Tensor wires, int[] slots, float[] weights, int n, int k, int levels=127, "
        "Tensor? out=None, bool accumulate=False) -> Tensor");
}

TORCH_LIBRARY_IMPL(flcodec, CUDA, m) {
  m.impl("stacked_encode", &stacked_encode);
  m.impl("stacked_decode", &stacked_decode);
  m.impl("stacked_decode_accumulate_", &stacked_decode_accumulate_);
  m.impl("topk_encode", &topk_encode);
  m.impl("sparse_decode", &sparse_decode);
  m.impl("quant_norm", &quant_norm);
  m.impl("quant_encode", &quant_encode);
  m.impl("quant_decode", &quant_decode);
  m.impl("natural_encode", &natural_encode);
  m.impl("natural_decode", &natural_decode);
  m.impl("weighted_sum_", &weighted_sum_);
  m.impl("fedopt_step_", &fedopt_step_);
  m.impl("model_fold_", &model_fold_);
  m.impl("delta_flatten", &delta_flatten);
  m.impl("feddr_combine_", &feddr_combine_);
  m.impl("stacked_encode_delta", &stacked_encode_delta);
  m.impl("quant_encode_auto", &quant_encode_auto);
  m.impl("adaptive_random", &adaptive_random);
  m.impl("stacked_encode_wire", &stacked_encode_wire);
  m.impl("stacked_encode_batch_wire", &stacked_encode_batch_wire);
  m.impl("stacked_fold_wires", &stacked_fold_wires);
}

TORCH_LIBRARY_IMPL(flcodec, Meta, m) {
  m.impl("stacked_encode", &stacked_encode_meta);
  m.impl("stacked_decode", &stacked_decode_meta);
  m.impl("topk_encode", &topk_encode_meta);
  m.impl("sparse_decode", &sparse_decode_meta);
  m.impl("quant_norm", &quant_norm_meta);
  m.impl("quant_encode", &quant_encode_meta);
  m.impl("quant_decode", &quant_decode_meta);
  m.impl("natural_encode", &natural_encode_meta);
  m.impl("natural_decode", &natural_decode_meta);
  m.impl("delta_flatten", &delta_flatten_meta);
  m.impl("stacked_encode_delta", &stacked_encode_delta_meta);
  m.impl("quant_encode_auto", &quant_encode_auto_meta);
  m.impl("adaptive_random", &adaptive_random_meta);
  m.impl("stacked_encode_wire", &stacked_encode_wire_meta);
  m.impl("stacked_encode_batch_wire", &stacked_encode_batch_wire_meta);
  m.impl("stacked_fold_wires", &stacked_fold_wires_meta);
}

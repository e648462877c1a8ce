// pyfold.cpp — `fl_sim_amd._flcfold.model_fold`: the server's whole-model fold (flc_model_fold) called straight from
// Python lists of tensors, for the per-round host path of FedOptServer.update / avg_parameters / add_parameters /
// update_gradients (_fedopt.py:196-240, nodes.py:1116-1180); `server_fold`, the same for FedDyn's and pFedMe's server
// updates (flc_model_fold_server); `avg_and_gradients`, the variance-reduced servers' avg_parameters + update_gradients
// (flc_avg_and_gradients); `stacked_delta_record`, a client's compressed message (flc_stacked_encode_delta into a wire
// record + flc_delta_count_nonzero_at).
//
// At configs[0] (cnn_femmist_tiny: 8 tensors, 10 clients) the kernel takes ~9 us, but going through the dispatcher
// (torch.ops.flcodec.model_fold_) cost ~14 us of host time: every tensor of the 96 in the call is boxed into an IValue
// list and unboxed again.  Here each Python tensor object is unpacked in place (THPVariable_Unpack, no refcount or
// IValue traffic), checked (HIP device, fp32, contiguous, sizes) and its pointer written into the table the C ABI
// takes; more than 16 messages are folded in chained launches (init mode 2 after the first launch, the optimizer
// step fused into the last one — the same fmaf chain as one launch).  Nothing is launched before every tensor of
// the call has passed its checks.  Errors: TypeError for a tensor the fold does not take (the caller then moves
// messages or folds per tensor), ValueError for mismatched sizes or counts.
//
// `alias(host_tensor, device_index)`: a HIP-device tensor over the same memory as a pinned host tensor, for the host
// server's zero-copy staging (hoststage.py): pinned host memory is mapped into every device's address space at the
// same address (checked here with hipPointerGetAttributes before the alias is made), so the fold kernels read and write
// the server's host tensors in place over PCIe.  The alias keeps the host storage alive.
#include <Python.h>
#include <torch/csrc/autograd/python_variable.h>
#include <c10/hip/HIPStream.h>
#include <ATen/ATen.h>

#include <vector>

#include "flcodec.h"

namespace {

constexpr int kMaxSrc = 16;  // messages per flc_model_fold launch

PyObject* type_error(const char* msg) {
  PyErr_SetString(PyExc_TypeError, msg);
  return nullptr;
}
PyObject* value_error(const char* msg) {
  PyErr_SetString(PyExc_ValueError, msg);
  return nullptr;
}

// a contiguous fp32 tensor on HIP device `dev` (-1: any HIP device, returned in *dev); nullptr if not one
const at::Tensor* usable(PyObject* o, int* dev) {
  if (!THPVariable_Check(o)) return nullptr;
  const at::Tensor& t = THPVariable_Unpack(o);
  if (!t.is_cuda() || t.scalar_type() != at::kFloat || !t.is_contiguous()) return nullptr;
  const int d = t.get_device();
  if (*dev < 0) *dev = d;
  else if (d != *dev) return nullptr;
  return &t;
}

// model_fold(dsts, msgs, key, weights, init_mode, beta, theta, v, opt, lr, beta2, tau)
//   dsts: sequence of model tensors (accumulators); msgs: sequence of messages, each a sequence of tensors or (key
//   not None) a mapping holding one under `key`; weights: one float per message; theta / v: sequences or None
PyObject* model_fold(PyObject*, PyObject* args) {
  PyObject *dsts, *msgs, *key, *weights, *theta, *v;
  int init_mode, opt;
  double beta, lr, beta2, tau;
  if (!PyArg_ParseTuple(args, "OOOOidOOiddd", &dsts, &msgs, &key, &weights, &init_mode, &beta, &theta, &v, &opt, &lr,
                        &beta2, &tau))
    return nullptr;
  PyObject* fd = PySequence_Fast(dsts, "dsts must be a sequence of tensors");
  if (!fd) return nullptr;
  PyObject* fm = PySequence_Fast(msgs, "messages must be a sequence");
  if (!fm) {
    Py_DECREF(fd);
    return nullptr;
  }
  PyObject* fw = PySequence_Fast(weights, "weights must be a sequence of floats");
  if (!fw) {
    Py_DECREF(fd);
    Py_DECREF(fm);
    return nullptr;
  }
  std::vector<PyObject*> keep = {fd, fm, fw};
  auto done = [&](PyObject* r) {
    for (PyObject* o : keep) Py_XDECREF(o);
    return r;
  };
  const Py_ssize_t nt = PySequence_Fast_GET_SIZE(fd), ns = PySequence_Fast_GET_SIZE(fm);
  if (PySequence_Fast_GET_SIZE(fw) != ns) return done(value_error("one weight per message"));
  if (nt == 0) return done((Py_INCREF(Py_None), Py_None));
  int dev = -1;
  std::vector<float*> dp(nt), tp, vp;
  std::vector<int64_t> sz(nt);
  PyObject** di = PySequence_Fast_ITEMS(fd);
  for (Py_ssize_t t = 0; t < nt; ++t) {
    const at::Tensor* a = usable(di[t], &dev);
    if (!a) return done(type_error("model tensors must be contiguous fp32 HIP tensors on one device"));
    dp[t] = a->data_ptr<float>();
    sz[t] = a->numel();
  }
  for (int which = 0; which < 2; ++which) {  // theta, v
    PyObject* src = which == 0 ? theta : v;
    if (src == Py_None) continue;
    PyObject* f = PySequence_Fast(src, "theta / v must be sequences of tensors");
    if (!f) return done(nullptr);
    keep.push_back(f);
    if (PySequence_Fast_GET_SIZE(f) != nt) return done(value_error("theta / v need one tensor per model tensor"));
    std::vector<float*>& out = which == 0 ? tp : vp;
    out.resize(nt);
    PyObject** it = PySequence_Fast_ITEMS(f);
    for (Py_ssize_t t = 0; t < nt; ++t) {
      const at::Tensor* a = usable(it[t], &dev);
      if (!a) return done(type_error("theta / v tensors must be contiguous fp32 HIP tensors on the model's device"));
      if (a->numel() != sz[t]) return done(value_error("theta / v must match the model tensors' sizes"));
      out[t] = a->data_ptr<float>();
    }
  }
  std::vector<const float*> sp((size_t)ns * nt);
  std::vector<float> w(ns);
  PyObject** mi = PySequence_Fast_ITEMS(fm);
  PyObject** wi = PySequence_Fast_ITEMS(fw);
  for (Py_ssize_t m = 0; m < ns; ++m) {
    const double wd = PyFloat_AsDouble(wi[m]);
    if (wd == -1.0 && PyErr_Occurred()) return done(nullptr);
    w[m] = (float)wd;  // (rounded to fp32 at the boundary, as torch's add_(alpha=...) does)
    PyObject* msg = mi[m];
    if (key != Py_None) {
      msg = PyObject_GetItem(msg, key);  // (new reference)
      if (!msg) return done(nullptr);
      keep.push_back(msg);
    }
    PyObject* f = PySequence_Fast(msg, "a message is a sequence of tensors");
    if (!f) return done(nullptr);
    keep.push_back(f);
    if (PySequence_Fast_GET_SIZE(f) != nt) return done(value_error("every message has one tensor per model tensor"));
    PyObject** it = PySequence_Fast_ITEMS(f);
    for (Py_ssize_t t = 0; t < nt; ++t) {
      const at::Tensor* a = usable(it[t], &dev);
      if (!a) return done(type_error("message tensors must be contiguous fp32 HIP tensors on the model's device"));
      if (a->numel() != sz[t]) return done(value_error("message tensors must match the model tensors' sizes"));
      sp[(size_t)m * nt + t] = a->data_ptr<float>();
    }
  }
  void* st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
  int rc = FLC_OK;
  Py_BEGIN_ALLOW_THREADS
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  Py_ssize_t m0 = 0;
  do {  // chained launches of <= 16 messages: the optimizer step with the last one only
    const Py_ssize_t cnt = ns - m0 < kMaxSrc ? ns - m0 : kMaxSrc;
    const bool last = m0 + cnt >= ns;
    rc = flc_model_fold(dp.data(), sp.data() + (size_t)m0 * nt, w.data() + m0, (int)cnt, sz.data(), (int)nt,
                        m0 == 0 ? init_mode : 2, (float)beta, last && !tp.empty() ? tp.data() : nullptr,
                        last && !vp.empty() ? vp.data() : nullptr, last ? opt : FLC_OPT_AVG, lr, beta2, tau, st);
    m0 += cnt;
  } while (rc == FLC_OK && m0 < ns);
  if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  Py_END_ALLOW_THREADS
  if (rc != FLC_OK) {
    PyErr_Format(PyExc_RuntimeError, "flc_model_fold failed with status %d: %s", rc, flc_last_error());
    return done(nullptr);
  }
  return done((Py_INCREF(Py_None), Py_None));
}

// server_fold(theta, aux, msgs, key, weights, kind, fold, init_mode, inertia, c): flc_model_fold_server (FedDyn's h
// fold + average, pFedMe's average + blend: feddyn/_feddyn.py:172-184, pfedme/_pfedme.py:166-175) on Python lists, at
// most 16 messages (the caller chains longer lists).  The same checks as model_fold, the same errors.
PyObject* server_fold(PyObject*, PyObject* args) {
  PyObject *theta, *aux, *msgs, *key, *weights;
  int kind, fold, init_mode;
  double inertia, c;
  if (!PyArg_ParseTuple(args, "OOOOOiiidd", &theta, &aux, &msgs, &key, &weights, &kind, &fold, &init_mode, &inertia,
                        &c))
    return nullptr;
  std::vector<PyObject*> keep;
  auto done = [&](PyObject* r) {
    for (PyObject* o : keep) Py_XDECREF(o);
    return r;
  };
  PyObject* ft = PySequence_Fast(theta, "theta must be a sequence of tensors");
  if (!ft) return nullptr;
  keep.push_back(ft);
  PyObject* fa = PySequence_Fast(aux, "aux must be a sequence of tensors");
  if (!fa) return done(nullptr);
  keep.push_back(fa);
  PyObject* fm = PySequence_Fast(msgs, "messages must be a sequence");
  if (!fm) return done(nullptr);
  keep.push_back(fm);
  PyObject* fw = PySequence_Fast(weights, "weights must be a sequence of floats");
  if (!fw) return done(nullptr);
  keep.push_back(fw);
  const Py_ssize_t nt = PySequence_Fast_GET_SIZE(ft), ns = PySequence_Fast_GET_SIZE(fm);
  if (PySequence_Fast_GET_SIZE(fw) != ns) return done(value_error("one weight per message"));
  if (PySequence_Fast_GET_SIZE(fa) != nt) return done(value_error("one aux tensor per model tensor"));
  if (ns > kMaxSrc) return done(value_error("server_fold takes at most 16 messages"));
  if (nt == 0) return done((Py_INCREF(Py_None), Py_None));
  int dev = -1;
  std::vector<float*> tp(nt), ap(nt);
  std::vector<int64_t> sz(nt);
  PyObject** ti = PySequence_Fast_ITEMS(ft);
  PyObject** ai = PySequence_Fast_ITEMS(fa);
  for (Py_ssize_t t = 0; t < nt; ++t) {
    const at::Tensor* a = usable(ti[t], &dev);
    if (!a) return done(type_error("model tensors must be contiguous fp32 HIP tensors on one device"));
    tp[t] = a->data_ptr<float>();
    sz[t] = a->numel();
    const at::Tensor* b = usable(ai[t], &dev);
    if (!b) return done(type_error("aux tensors must be contiguous fp32 HIP tensors on the model's device"));
    if (b->numel() != sz[t]) return done(value_error("aux tensors must match the model tensors' sizes"));
    ap[t] = b->data_ptr<float>();
  }
  std::vector<const float*> sp((size_t)(ns > 0 ? ns : 1) * nt);
  std::vector<float> w(ns > 0 ? ns : 1);
  PyObject** mi = PySequence_Fast_ITEMS(fm);
  PyObject** wi = PySequence_Fast_ITEMS(fw);
  for (Py_ssize_t m = 0; m < ns; ++m) {
    const double wd = PyFloat_AsDouble(wi[m]);
    if (wd == -1.0 && PyErr_Occurred()) return done(nullptr);
    w[m] = (float)wd;
    PyObject* msg = mi[m];
    if (key != Py_None) {
      msg = PyObject_GetItem(msg, key);
      if (!msg) return done(nullptr);
      keep.push_back(msg);
    }
    PyObject* f = PySequence_Fast(msg, "a message is a sequence of tensors");
    if (!f) return done(nullptr);
    keep.push_back(f);
    if (PySequence_Fast_GET_SIZE(f) != nt) return done(value_error("every message has one tensor per model tensor"));
    PyObject** it = PySequence_Fast_ITEMS(f);
    for (Py_ssize_t t = 0; t < nt; ++t) {
      const at::Tensor* a = usable(it[t], &dev);
      if (!a) return done(type_error("message tensors must be contiguous fp32 HIP tensors on the model's device"));
      if (a->numel() != sz[t]) return done(value_error("message tensors must match the model tensors' sizes"));
      sp[(size_t)m * nt + t] = a->data_ptr<float>();
    }
  }
  void* st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
  int rc = FLC_OK;
  Py_BEGIN_ALLOW_THREADS
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  rc = flc_model_fold_server(tp.data(), ap.data(), sp.data(), w.data(), (int)ns, sz.data(), (int)nt, kind, fold,
                             init_mode, (float)inertia, c, st);
  if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  Py_END_ALLOW_THREADS
  if (rc != FLC_OK) {
    PyErr_Format(PyExc_RuntimeError, "flc_model_fold_server failed with status %d: %s", rc, flc_last_error());
    return done(nullptr);
  }
  return done((Py_INCREF(Py_None), Py_None));
}

// avg_and_gradients(params, grads, msgs, w_params, w_grads, inertia[, set_grad]): flc_avg_and_gradients
// (avg_parameters then update_gradients over the same messages, nodes.py:1134-1180) on Python lists: `params` folded
// in place, `grads` (one per parameter, same sizes) written from +0; every message a mapping with "parameters" and
// "gradients".  `grads` None: the gradients go into one new flat fp32 buffer on the model's device, returned as
// (list of per-parameter views, flat buffer), and with `set_grad` each parameter's `.grad` is set to its view (as
// update_gradients' `mp.grad = ...`) — the per-update Python work of the device-resident variance-reduced servers
// (views, `.grad` setters) done here.  The same checks and errors as model_fold, all before anything is allocated or
// launched; any number of messages (the C call chains them).
PyObject* avg_and_gradients(PyObject*, PyObject* args) {
  PyObject *params, *grads, *msgs, *wpar, *wgrd;
  double inertia;
  int set_grad = 0;
  if (!PyArg_ParseTuple(args, "OOOOOd|p", &params, &grads, &msgs, &wpar, &wgrd, &inertia, &set_grad)) return nullptr;
  std::vector<PyObject*> keep;
  auto done = [&](PyObject* r) {
    for (PyObject* o : keep) Py_XDECREF(o);
    return r;
  };
  const bool alloc = grads == Py_None;
  PyObject* seqs[5] = {params, alloc ? params : grads, msgs, wpar, wgrd};
  PyObject* f[5];
  for (int i = 0; i < 5; ++i) {
    f[i] = PySequence_Fast(seqs[i], "avg_and_gradients takes sequences");
    if (!f[i]) return done(nullptr);
    keep.push_back(f[i]);
  }
  const Py_ssize_t nt = PySequence_Fast_GET_SIZE(f[0]), ns = PySequence_Fast_GET_SIZE(f[2]);
  if (PySequence_Fast_GET_SIZE(f[1]) != nt) return done(value_error("one gradient buffer per parameter"));
  if (PySequence_Fast_GET_SIZE(f[3]) != ns || PySequence_Fast_GET_SIZE(f[4]) != ns)
    return done(value_error("one weight of each kind per message"));
  if (ns == 0) return done(value_error("avg_and_gradients needs at least one message"));
  if (nt == 0) return done((Py_INCREF(Py_None), Py_None));
  int dev = -1;
  std::vector<float*> pp(nt), gp(nt);
  std::vector<int64_t> sz(nt);
  std::vector<const at::Tensor*> pt(nt);
  PyObject** pi = PySequence_Fast_ITEMS(f[0]);
  PyObject** gi = PySequence_Fast_ITEMS(f[1]);
  for (Py_ssize_t t = 0; t < nt; ++t) {
    const at::Tensor* a = usable(pi[t], &dev);
    if (!a) return done(type_error("model tensors must be contiguous fp32 HIP tensors on one device"));
    pt[t] = a;
    pp[t] = a->data_ptr<float>();
    sz[t] = a->numel();
    if (alloc) continue;
    const at::Tensor* b = usable(gi[t], &dev);
    if (!b) return done(type_error("gradient buffers must be contiguous fp32 HIP tensors on the model's device"));
    if (b->numel() != sz[t]) return done(value_error("gradient buffers must match the model tensors' sizes"));
    gp[t] = b->data_ptr<float>();
  }
  std::vector<const float*> ps((size_t)ns * nt), gs((size_t)ns * nt);
  std::vector<float> wp(ns), wg(ns);
  PyObject** mi = PySequence_Fast_ITEMS(f[2]);
  PyObject** wpi = PySequence_Fast_ITEMS(f[3]);
  PyObject** wgi = PySequence_Fast_ITEMS(f[4]);
  static PyObject* const keys[2] = {PyUnicode_InternFromString("parameters"), PyUnicode_InternFromString("gradients")};
  for (Py_ssize_t m = 0; m < ns; ++m) {
    const double a = PyFloat_AsDouble(wpi[m]), b = PyFloat_AsDouble(wgi[m]);
    if (PyErr_Occurred()) return done(nullptr);
    wp[m] = (float)a;
    wg[m] = (float)b;
    for (int k = 0; k < 2; ++k) {
      PyObject* v = PyObject_GetItem(mi[m], keys[k]);
      if (!v) return done(nullptr);
      keep.push_back(v);
      PyObject* fv = PySequence_Fast(v, "a message's parameters / gradients are sequences of tensors");
      if (!fv) return done(nullptr);
      keep.push_back(fv);
      if (PySequence_Fast_GET_SIZE(fv) != nt) return done(value_error("every message has one tensor per model tensor"));
      PyObject** it = PySequence_Fast_ITEMS(fv);
      std::vector<const float*>& out = k == 0 ? ps : gs;
      for (Py_ssize_t t = 0; t < nt; ++t) {
        const at::Tensor* s = usable(it[t], &dev);
        if (!s) return done(type_error("message tensors must be contiguous fp32 HIP tensors on the model's device"));
        if (s->numel() != sz[t]) return done(value_error("message tensors must match the model tensors' sizes"));
        out[(size_t)m * nt + t] = s->data_ptr<float>();
      }
    }
  }
  // (every tensor checked: the gradient buffer, when asked for, is allocated now)
  at::Tensor flat;
  std::vector<at::Tensor> gv;
  if (alloc) {
    int64_t total = 0;
    for (Py_ssize_t t = 0; t < nt; ++t) total += sz[t];
    try {
      flat = at::empty({total > 0 ? total : 1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
    } catch (const std::exception& e) {
      PyErr_SetString(PyExc_RuntimeError, e.what());
      return done(nullptr);
    }
    gv.reserve(nt);
    int64_t off = 0;
    for (Py_ssize_t t = 0; t < nt; ++t) {
      gv.push_back(flat.narrow(0, off, sz[t]).view(pt[t]->sizes()));
      gp[t] = flat.data_ptr<float>() + off;
      off += sz[t];
    }
  }
  void* st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
  int rc = FLC_OK;
  Py_BEGIN_ALLOW_THREADS
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  rc = flc_avg_and_gradients(pp.data(), gp.data(), ps.data(), gs.data(), wp.data(), wg.data(), (int)ns, sz.data(),
                             (int)nt, (float)inertia, st);
  if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  Py_END_ALLOW_THREADS
  if (rc != FLC_OK) {
    PyErr_Format(PyExc_RuntimeError, "flc_avg_and_gradients failed with status %d: %s", rc, flc_last_error());
    return done(nullptr);
  }
  if (!alloc) return done((Py_INCREF(Py_None), Py_None));
  PyObject* lst = PyList_New(nt);
  if (!lst) return done(nullptr);
  for (Py_ssize_t t = 0; t < nt; ++t) {
    if (set_grad) pt[t]->mutable_grad() = gv[t];  // (update_gradients' `mp.grad = ...`: same device, dtype, sizes)
    PyObject* w = THPVariable_Wrap(gv[t]);
    if (!w) {
      Py_DECREF(lst);
      return done(nullptr);
    }
    PyList_SET_ITEM(lst, t, w);
  }
  PyObject* fl = THPVariable_Wrap(flat);
  if (!fl) {
    Py_DECREF(lst);
    return done(nullptr);
  }
  return done(Py_BuildValue("(NN)", lst, fl));
}

// a contiguous HIP tensor of `dt` on device `dev` (-1: any, returned); nullptr if not one
const at::Tensor* usable_as(PyObject* o, at::ScalarType dt, int* dev) {
  if (!THPVariable_Check(o)) return nullptr;
  const at::Tensor& t = THPVariable_Unpack(o);
  if (!t.is_cuda() || t.scalar_type() != dt || !t.is_contiguous()) return nullptr;
  const int d = t.get_device();
  if (*dev < 0) *dev = d;
  else if (d != *dev) return nullptr;
  return &t;
}

// stacked_delta_record(local, global, k, levels, seed, counter, record, count, ws): FedOptClient.communicate's delta
// (_fedopt.py:295-308) through the stacked pipeline in one C call — flc_stacked_encode_delta of cat(local - global)
// into the packed wire record `record` (a contiguous uint8 HIP tensor of at least flc_stacked_wire_layout(n, k) bytes,
// 16-B aligned; the delta is formed in the encoder's read), then, with `count` (an int64 HIP tensor), the dithering
// stage's send count (flc_delta_count_nonzero_at over the kept entries).  `ws`: the encoder's workspace (uint8).  The
// same checks as model_fold: TypeError for a tensor the encoder does not take (the caller converts and retries),
// ValueError for sizes.
PyObject* stacked_delta_record(PyObject*, PyObject* args) {
  PyObject *loc, *glo, *record, *count, *wso;
  long long k;
  int levels;
  unsigned long long seed, counter;
  if (!PyArg_ParseTuple(args, "OOLiKKOOO", &loc, &glo, &k, &levels, &seed, &counter, &record, &count, &wso))
    return nullptr;
  std::vector<PyObject*> keep;
  auto done = [&](PyObject* r) {
    for (PyObject* o : keep) Py_XDECREF(o);
    return r;
  };
  PyObject* fl = PySequence_Fast(loc, "local must be a sequence of tensors");
  if (!fl) return nullptr;
  keep.push_back(fl);
  PyObject* fg = PySequence_Fast(glo, "global must be a sequence of tensors");
  if (!fg) return done(nullptr);
  keep.push_back(fg);
  const Py_ssize_t m = PySequence_Fast_GET_SIZE(fl);
  if (m < 1 || PySequence_Fast_GET_SIZE(fg) != m) return done(value_error("one global tensor per local tensor, at least one"));
  int dev = -1;
  std::vector<const float*> lp(m), gp(m);
  std::vector<int64_t> sz(m);
  PyObject** li = PySequence_Fast_ITEMS(fl);
  PyObject** gi = PySequence_Fast_ITEMS(fg);
  int64_t n = 0;
  for (Py_ssize_t t = 0; t < m; ++t) {
    const at::Tensor* a = usable(li[t], &dev);
    const at::Tensor* b = usable(gi[t], &dev);
    if (!a || !b) return done(type_error("local / global tensors must be contiguous fp32 HIP tensors on one device"));
    if (a->numel() != b->numel()) return done(value_error("local and global tensors must have matching sizes"));
    lp[t] = a->data_ptr<float>();
    gp[t] = b->data_ptr<float>();
    sz[t] = a->numel();
    n += sz[t];
  }
  const at::Tensor* rec = usable_as(record, at::kByte, &dev);
  if (!rec) return done(type_error("the record must be a contiguous uint8 HIP tensor on the tensors' device"));
  int64_t off[4] = {0, 0, 0, 0};  // norm, idx, codes, tiles
  const size_t stride = flc_stacked_wire_layout(n, k, off);
  uint8_t* rp = rec->data_ptr<uint8_t>();
  if (stride == 0 || (size_t)rec->numel() < stride || reinterpret_cast<uintptr_t>(rp) % 16 != 0)
    return done(value_error("the record is smaller than the wire layout or not 16-B aligned"));
  int64_t* cp = nullptr;
  if (count != Py_None) {
    const at::Tensor* c = usable_as(count, at::kLong, &dev);
    if (!c || c->numel() < 1) return done(type_error("count must be an int64 HIP tensor on the tensors' device"));
    cp = c->data_ptr<int64_t>();
  }
  const at::Tensor* ws = usable_as(wso, at::kByte, &dev);
  if (!ws) return done(type_error("ws must be a contiguous uint8 HIP tensor on the tensors' device"));
  void* st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
  int32_t* idx = reinterpret_cast<int32_t*>(rp + off[1]);
  int rc = FLC_OK;
  const char* what = "flc_stacked_encode_delta";
  Py_BEGIN_ALLOW_THREADS
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  rc = flc_stacked_encode_delta(lp.data(), gp.data(), sz.data(), (int)m, k, levels, seed, counter, idx, rp + off[2],
                                reinterpret_cast<float*>(rp + off[0]), reinterpret_cast<uint32_t*>(rp + off[3]),
                                ws->data_ptr(), (size_t)ws->numel(), st);
  if (rc == FLC_OK && cp) {
    what = "flc_delta_count_nonzero_at";
    rc = flc_delta_count_nonzero_at(lp.data(), gp.data(), sz.data(), (int)m, idx, k, cp, st);
  }
  if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  Py_END_ALLOW_THREADS
  if (rc != FLC_OK) {
    PyErr_Format(PyExc_RuntimeError, "%s failed with status %d: %s", what, rc, flc_last_error());
    return done(nullptr);
  }
  return done((Py_INCREF(Py_None), Py_None));
}

// delta_flat(local, global): a new flat fp32 tensor = cat(local_t - global_t) (flc_delta_flatten) on the tensors'
// device — the deferred compressed message's snapshot of its delta (compressed.py).  TypeError (nothing allocated)
// for a tensor that is not a contiguous fp32 HIP tensor of one device.
PyObject* delta_flat(PyObject*, PyObject* args) {
  PyObject *loc, *glo;
  if (!PyArg_ParseTuple(args, "OO", &loc, &glo)) return nullptr;
  std::vector<PyObject*> keep;
  auto done = [&](PyObject* r) {
    for (PyObject* o : keep) Py_XDECREF(o);
    return r;
  };
  PyObject* fl = PySequence_Fast(loc, "local must be a sequence of tensors");
  if (!fl) return nullptr;
  keep.push_back(fl);
  PyObject* fg = PySequence_Fast(glo, "global must be a sequence of tensors");
  if (!fg) return done(nullptr);
  keep.push_back(fg);
  const Py_ssize_t m = PySequence_Fast_GET_SIZE(fl);
  if (m < 1 || PySequence_Fast_GET_SIZE(fg) != m) return done(value_error("one global tensor per local tensor, at least one"));
  int dev = -1;
  std::vector<const float*> lp(m), gp(m);
  std::vector<int64_t> sz(m);
  PyObject** li = PySequence_Fast_ITEMS(fl);
  PyObject** gi = PySequence_Fast_ITEMS(fg);
  int64_t n = 0;
  for (Py_ssize_t t = 0; t < m; ++t) {
    const at::Tensor* a = usable(li[t], &dev);
    const at::Tensor* b = usable(gi[t], &dev);
    if (!a || !b) return done(type_error("local / global tensors must be contiguous fp32 HIP tensors on one device"));
    if (a->numel() != b->numel()) return done(value_error("local and global tensors must have matching sizes"));
    lp[t] = a->data_ptr<float>();
    gp[t] = b->data_ptr<float>();
    sz[t] = a->numel();
    n += sz[t];
  }
  at::Tensor out;
  try {
    out = at::empty({n > 0 ? n : 1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return done(nullptr);
  }
  if (n == 0) out = out.narrow(0, 0, 0);
  void* st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
  int rc = FLC_OK;
  float* op = out.data_ptr<float>();
  Py_BEGIN_ALLOW_THREADS
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  rc = flc_delta_flatten(lp.data(), gp.data(), sz.data(), (int)m, op, st);
  if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  Py_END_ALLOW_THREADS
  if (rc != FLC_OK) {
    PyErr_Format(PyExc_RuntimeError, "flc_delta_flatten failed with status %d: %s", rc, flc_last_error());
    return done(nullptr);
  }
  return done(THPVariable_Wrap(out));
}

// stacked_records_batch(flats, seeds, counter, k, levels, records, counts, ws): the deferred messages of a round in
// one C call — flc_stacked_encode_batch of the flat deltas into rows of the [C, >= stride] record block (row c equals
// client c's one-message record), then flc_count_nonzero_at_batch of each delta at its kept indices into counts[c].
PyObject* stacked_records_batch(PyObject*, PyObject* args) {
  PyObject *flats, *seeds, *recs, *counts, *wso;
  unsigned long long counter;
  long long k;
  int levels;
  if (!PyArg_ParseTuple(args, "OOKLiOOO", &flats, &seeds, &counter, &k, &levels, &recs, &counts, &wso)) return nullptr;
  std::vector<PyObject*> keep;
  auto done = [&](PyObject* r) {
    for (PyObject* o : keep) Py_XDECREF(o);
    return r;
  };
  PyObject* seqs[3] = {flats, seeds, counts};
  PyObject* f[3];
  for (int i = 0; i < 3; ++i) {
    f[i] = PySequence_Fast(seqs[i], "stacked_records_batch takes sequences");
    if (!f[i]) return done(nullptr);
    keep.push_back(f[i]);
  }
  const Py_ssize_t C = PySequence_Fast_GET_SIZE(f[0]);
  if (C < 1 || PySequence_Fast_GET_SIZE(f[1]) != C || PySequence_Fast_GET_SIZE(f[2]) != C)
    return done(value_error("one seed and one count per client, at least one client"));
  int dev = -1;
  int64_t n = -1;
  std::vector<const float*> xp(C);
  std::vector<uint64_t> sd(C);
  std::vector<int64_t*> cp(C);
  PyObject** xi = PySequence_Fast_ITEMS(f[0]);
  PyObject** si = PySequence_Fast_ITEMS(f[1]);
  PyObject** ci = PySequence_Fast_ITEMS(f[2]);
  for (Py_ssize_t c = 0; c < C; ++c) {
    const at::Tensor* x = usable(xi[c], &dev);
    if (!x) return done(type_error("flat deltas must be contiguous fp32 HIP tensors on one device"));
    if (n < 0) n = x->numel();
    if (x->numel() != n) return done(value_error("flat deltas must all have one size"));
    xp[c] = x->data_ptr<float>();
    sd[c] = (uint64_t)PyLong_AsUnsignedLongLongMask(si[c]);
    if (PyErr_Occurred()) return done(nullptr);
    const at::Tensor* ct = usable_as(ci[c], at::kLong, &dev);
    if (!ct || ct->numel() < 1) return done(type_error("counts must be int64 HIP tensors on the deltas' device"));
    cp[c] = ct->data_ptr<int64_t>();
  }
  int64_t off[4] = {0, 0, 0, 0};  // norm, idx, codes, tiles
  const size_t stride = flc_stacked_wire_layout(n, k, off);
  if (stride == 0) return done(value_error("bad wire shape"));
  if (!THPVariable_Check(recs)) return done(type_error("records must be a uint8 HIP tensor"));
  const at::Tensor& rb = THPVariable_Unpack(recs);
  if (!rb.is_cuda() || rb.get_device() != dev || rb.scalar_type() != at::kByte || rb.dim() != 2 || !rb.is_contiguous() ||
      rb.size(0) != C || rb.size(1) < (int64_t)stride || rb.size(1) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(rb.data_ptr()) % 16 != 0)
    return done(value_error("records must be a contiguous [clients, >= stride] uint8 block (16-B rows) on the device"));
  const at::Tensor* ws = usable_as(wso, at::kByte, &dev);
  if (!ws) return done(type_error("ws must be a contiguous uint8 HIP tensor on the deltas' device"));
  uint8_t* base = rb.data_ptr<uint8_t>();
  const int64_t rs = rb.size(1);
  std::vector<int32_t*> ip(C);
  std::vector<uint8_t*> kp(C);
  std::vector<float*> np(C);
  std::vector<uint32_t*> tp(C);
  std::vector<const int32_t*> cip(C);
  for (Py_ssize_t c = 0; c < C; ++c) {
    uint8_t* r = base + c * rs;
    np[c] = reinterpret_cast<float*>(r + off[0]);
    ip[c] = reinterpret_cast<int32_t*>(r + off[1]);
    cip[c] = ip[c];
    kp[c] = r + off[2];
    tp[c] = reinterpret_cast<uint32_t*>(r + off[3]);
  }
  void* st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
  int rc = FLC_OK;
  const char* what = "flc_stacked_encode_batch";
  Py_BEGIN_ALLOW_THREADS
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  rc = flc_stacked_encode_batch(xp.data(), (int)C, n, k, levels, sd.data(), counter, ip.data(), kp.data(), np.data(),
                                tp.data(), ws->data_ptr(), (size_t)ws->numel(), st);
  if (rc == FLC_OK) {
    what = "flc_count_nonzero_at_batch";
    rc = flc_count_nonzero_at_batch(xp.data(), cip.data(), (int)C, n, k, cp.data(), st);
  }
  if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  Py_END_ALLOW_THREADS
  if (rc != FLC_OK) {
    PyErr_Format(PyExc_RuntimeError, "%s failed with status %d: %s", what, rc, flc_last_error());
    return done(nullptr);
  }
  return done((Py_INCREF(Py_None), Py_None));
}

// fold_records(records, weights, n, k, levels, delta, theta, v, beta0, opt, lr, beta2, tau): the server update of a
// round of stacked records (flc_fedopt_fold_records) on Python lists.  TypeError (nothing launched) when a tensor is
// not what the pass takes — the server tensors contiguous fp32 HIP tensors of one device summing to n, the records
// 16-B aligned uint8 tensors of at least the wire layout's bytes on that device — so the caller can take its other
// path; theta / v None: the fold alone / no second moment.
PyObject* fold_records(PyObject*, PyObject* args) {
  PyObject *recs, *weights, *delta, *theta, *v;
  long long n, k;
  int levels, opt;
  double beta0, lr, beta2, tau;
  if (!PyArg_ParseTuple(args, "OOLLiOOOdiddd", &recs, &weights, &n, &k, &levels, &delta, &theta, &v, &beta0, &opt, &lr,
                        &beta2, &tau))
    return nullptr;
  std::vector<PyObject*> keep;
  auto done = [&](PyObject* r) {
    for (PyObject* o : keep) Py_XDECREF(o);
    return r;
  };
  PyObject* seqs[3] = {recs, weights, delta};
  PyObject* f[3];
  for (int i = 0; i < 3; ++i) {
    f[i] = PySequence_Fast(seqs[i], "fold_records takes sequences");
    if (!f[i]) return done(nullptr);
    keep.push_back(f[i]);
  }
  const Py_ssize_t nr = PySequence_Fast_GET_SIZE(f[0]), nt = PySequence_Fast_GET_SIZE(f[2]);
  if (PySequence_Fast_GET_SIZE(f[1]) != nr) return done(value_error("one weight per record"));
  if (nr < 1 || nt < 1) return done(type_error("fold_records needs records and server tensors"));
  int dev = -1;
  std::vector<float*> dp(nt), tp, vp;
  std::vector<int64_t> sz(nt);
  int64_t total = 0;
  PyObject** di = PySequence_Fast_ITEMS(f[2]);
  for (Py_ssize_t t = 0; t < nt; ++t) {
    const at::Tensor* a = usable(di[t], &dev);
    if (!a) return done(type_error("server tensors must be contiguous fp32 HIP tensors on one device"));
    dp[t] = a->data_ptr<float>();
    sz[t] = a->numel();
    total += sz[t];
  }
  if (total != n) return done(type_error("the server tensors do not hold the records' element count"));
  for (int which = 0; which < 2; ++which) {
    PyObject* src = which == 0 ? theta : v;
    if (src == Py_None) continue;
    PyObject* fs = PySequence_Fast(src, "theta / v must be sequences of tensors");
    if (!fs) return done(nullptr);
    keep.push_back(fs);
    if (PySequence_Fast_GET_SIZE(fs) != nt) return done(type_error("theta / v need one tensor per server tensor"));
    std::vector<float*>& out = which == 0 ? tp : vp;
    out.resize(nt);
    PyObject** it = PySequence_Fast_ITEMS(fs);
    for (Py_ssize_t t = 0; t < nt; ++t) {
      const at::Tensor* a = usable(it[t], &dev);
      if (!a || a->numel() != sz[t]) return done(type_error("theta / v must match the server tensors"));
      out[t] = a->data_ptr<float>();
    }
  }
  int64_t off[4];
  const size_t stride = flc_stacked_wire_layout(n, k, off);
  if (stride == 0) return done(value_error("bad wire shape"));
  std::vector<const void*> rp(nr);
  std::vector<float> w(nr);
  PyObject** ri = PySequence_Fast_ITEMS(f[0]);
  PyObject** wi = PySequence_Fast_ITEMS(f[1]);
  for (Py_ssize_t c = 0; c < nr; ++c) {
    const at::Tensor* r = usable_as(ri[c], at::kByte, &dev);
    if (!r || (size_t)r->numel() < stride || reinterpret_cast<uintptr_t>(r->data_ptr()) % 16 != 0)
      return done(type_error("records must be 16-B aligned uint8 HIP tensors of the wire layout on the server's device"));
    rp[c] = r->data_ptr();
    const double wd = PyFloat_AsDouble(wi[c]);
    if (wd == -1.0 && PyErr_Occurred()) return done(nullptr);
    w[c] = (float)wd;
  }
  void* st = c10::hip::getCurrentHIPStream((c10::DeviceIndex)dev).stream();
  int rc = FLC_OK;
  Py_BEGIN_ALLOW_THREADS
  int cur = -1;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  rc = flc_fedopt_fold_records(rp.data(), w.data(), (int)nr, n, k, levels, dp.data(), tp.empty() ? nullptr : tp.data(),
                               vp.empty() ? nullptr : vp.data(), sz.data(), (int)nt, (float)beta0, opt, lr, beta2, tau,
                               st);
  if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  Py_END_ALLOW_THREADS
  if (rc != FLC_OK) {
    PyErr_Format(PyExc_RuntimeError, "flc_fedopt_fold_records failed with status %d: %s", rc, flc_last_error());
    return done(nullptr);
  }
  return done((Py_INCREF(Py_None), Py_None));
}

void release_storage(void* ctx) { delete static_cast<c10::Storage*>(ctx); }

// alias(host_tensor, device_index) -> tensor on cuda:device_index over the same bytes (see the header)
PyObject* alias(PyObject*, PyObject* args) {
  PyObject* o;
  int dev;
  if (!PyArg_ParseTuple(args, "Oi", &o, &dev)) return nullptr;
  if (!THPVariable_Check(o)) return type_error("alias takes a tensor");
  const at::Tensor& t = THPVariable_Unpack(o);
  if (!t.is_cpu() || !t.is_contiguous() || !t.is_pinned()) return type_error("alias takes a contiguous pinned host tensor");
  void* p = t.data_ptr();
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost || a.devicePointer != p) {
    (void)hipGetLastError();
    PyErr_SetString(PyExc_RuntimeError, "the pinned buffer is not mapped at its host address on the device");
    return nullptr;
  }
  const size_t nbytes = (size_t)t.numel() * t.element_size();
  auto* keep = new c10::Storage(t.storage());
  c10::DataPtr dp(p, keep, &release_storage, c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)dev));
  c10::Storage st(c10::Storage::use_byte_size_t(), nbytes, std::move(dp), /*allocator=*/nullptr, /*resizable=*/false);
  at::Tensor d = at::empty({0}, t.options().device(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)dev)).pinned_memory(false));
  d.set_(st, 0, t.sizes(), t.strides());
  return THPVariable_Wrap(d);
}

PyMethodDef kMethods[] = {
    {"model_fold", model_fold, METH_VARARGS,
     "model_fold(dsts, msgs, key, weights, init_mode, beta, theta, v, opt, lr, beta2, tau): flc_model_fold on Python "
     "lists of HIP tensors, launched on the current stream of the model's device"},
    {"server_fold", server_fold, METH_VARARGS,
     "server_fold(theta, aux, msgs, key, weights, kind, fold, init_mode, inertia, c): flc_model_fold_server (FedDyn / "
     "pFedMe) on Python lists of HIP tensors, at most 16 messages, on the current stream of the model's device"},
    {"avg_and_gradients", avg_and_gradients, METH_VARARGS,
     "avg_and_gradients(params, grads, msgs, w_params, w_grads, inertia[, set_grad]): flc_avg_and_gradients on Python "
     "lists of HIP "
     "tensors (messages: mappings with 'parameters' and 'gradients'), on the current stream of the model's device"},
    {"fold_records", fold_records, METH_VARARGS,
     "fold_records(records, weights, n, k, levels, delta, theta, v, beta0, opt, lr, beta2, tau): "
     "flc_fedopt_fold_records on Python lists"},
    {"delta_flat", delta_flat, METH_VARARGS,
     "delta_flat(local, global): a new flat fp32 tensor cat(local - global) (flc_delta_flatten) on the tensors' device"},
    {"stacked_records_batch", stacked_records_batch, METH_VARARGS,
     "stacked_records_batch(flats, seeds, counter, k, levels, records, counts, ws): flc_stacked_encode_batch into the "
     "rows of a record block, then flc_count_nonzero_at_batch into counts"},
    {"stacked_delta_record", stacked_delta_record, METH_VARARGS,
     "stacked_delta_record(local, global, k, levels, seed, counter, record, count, ws): flc_stacked_encode_delta into a "
     "packed wire record (+ flc_delta_count_nonzero_at into count) on the current stream of the tensors' device"},
    {"alias", alias, METH_VARARGS,
     "alias(host_tensor, device_index): a HIP-device tensor over a pinned host tensor's memory (zero-copy)"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_flcfold", nullptr, -1, kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__flcfold(void) { return PyModule_Create(&kModule); }

/*
 * flcodec.h — C ABI of the MI355X-native gradient codec + aggregation path for fl-sim.
 *
 * The reference (wenh06/fl-sim) has no native code and no FFI: its codec is the pure-Python class
 * `Compressor` (fl_sim/compressors/compressors.py:35-419) and its aggregation is a set of in-place
 * torch loops on the `Server` (fl_sim/nodes.py:1116-1180, fl_sim/algorithms/fedopt/_fedopt.py:196-265).
 * Every entry point below replaces one branch of those Python functions; the comment on each cites
 * the reference lines it stands in for.  INTEGRATION.md shows the ctypes binding a maintainer adds to
 * the reference (fl_sim_amd/_lib.py is that binding, shipped).
 *
 * Conventions (all entry points):
 *   - plain pointers and sizes, no framework types; every device pointer is HBM memory of the current
 *     HIP device, every `stream` is a hipStream_t passed as void* (NULL = the default stream);
 *   - the caller owns every buffer, including the workspace (`*_workspace_size` says how much);
 *     a workspace must be zero-filled once after allocation (flc_workspace_init) and may then be reused
 *     by any number of calls on the same stream (counters reset themselves in-kernel);
 *   - stream-ordered and asynchronous: nothing here synchronises the stream except the host-only RNG
 *     helpers and flc_probe_read; no allocation happens inside a call, so calls can be graph-captured;
 *   - the return value is a status code (FLC_OK = 0); flc_last_error() describes the last failure of
 *     the calling thread;
 *   - element counts are int64_t but a single vector must have fewer than 2^31 elements (index
 *     streams are int32, as the reference's argsort indices fit int32 below that size);
 *   - RNG: every stochastic codec takes (seed, counter) for the counter-based Philox4x32-10 stream
 *     ("philox" mode), or a device array `compat_u` of fp64 uniforms, one per consuming element in
 *     index order ("compat" mode: the exact uniforms Python's `random.random()` would have produced —
 *     see flc_mt_random_doubles).  compat_u == NULL selects philox mode.
 */
#ifndef FLCODEC_H_
#define FLCODEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLC_ABI_VERSION 1

enum flc_status {
  FLC_OK = 0,
  FLC_EINVAL = 1,       /* bad argument (sizes, levels, bits, null pointer) */
  FLC_EHIP = 2,         /* HIP runtime error */
  FLC_EWORKSPACE = 3,   /* workspace too small */
  FLC_EUNSUPPORTED = 4, /* valid request this build does not implement */
  FLC_ECOMM = 5         /* RCCL error, or RCCL could not be loaded */
};

/* dense quantizer families (compressors.py:327-404) */
enum flc_quant_kind {
  FLC_Q_STANDARD_DITHER = 0, /* levels i/s, i = 0..s          (compressors.py:154-182, 327-365) */
  FLC_Q_NATURAL_DITHER = 1   /* levels 0, 2^-(s-1), .., 1/2, 1 (compressors.py:191-221, 367-404) */
};
enum flc_norm_kind { FLC_NORM_INF = 0, FLC_NORM_L2 = 2 };

/* proximal step of FedDR's regularizer (regularizers.py:146-200) */
enum flc_prox_kind { FLC_PROX_NONE = 0, FLC_PROX_L1 = 1, FLC_PROX_SCALE = 2 };

/* server optimiser of FedOptServer.update (_fedopt.py:196-265) */
enum flc_fedopt_kind { FLC_OPT_AVG = 0, FLC_OPT_ADAGRAD = 1, FLC_OPT_YOGI = 2, FLC_OPT_ADAM = 3 };

/* ------------------------------------------------------------------ library */
int flc_abi_version(void);
const char* flc_last_error(void);
/* zero a freshly allocated workspace (once); stream-ordered */
int flc_workspace_init(void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ host RNG (compat mode)
 * Python's `random` and numpy's legacy `RandomState` are both MT19937.  These host functions advance
 * a state exported by `random.getstate()[1]` (624 words + position) or `np.random.get_state()`
 * (624 words, position) exactly as the interpreter would, so the caller can write the advanced state
 * back and the global streams stay in lock-step with the reference (misc.py:196-217 seeds them).  */

/* n draws of random.random() (compressors.py:277, 316, 349, 386) == legacy random_sample (res53) */
int flc_mt_random_doubles(uint32_t* mt_state624, int32_t* mt_pos, double* out, int64_t n);
/* np.random.shuffle(np.arange(D)) then [:K] (compressors.py:285-287): legacy Fisher-Yates with
 * masked-rejection random_interval; writes the first K entries of the shuffled permutation */
int flc_np_shuffle_prefix(uint32_t* mt_state624, int32_t* mt_pos, int64_t D, int64_t K, int32_t* out_idx);

/* ------------------------------------------------------------------ dense quantizer codec
 * x is a [rows, d] row-major fp32 batch: one client delta per row (rows = 1 for compressVector).
 * Wire format per row: one fp32 norm + a packed code stream of `bits` (2, 4 or 8) bits per element,
 *   code = sign << (bits-1) | level, level in 0..s (s < 2^(bits-1)); element i of the flat batch sits
 *   at bit offset i*bits of `codes` (little-endian within a byte).
 * A row whose norm is not finite is encoded as code 0 for x == 0 and code 1 otherwise; it decodes to
 *   +0 / NaN, which is what the reference produces for such rows. */
size_t flc_quant_workspace_size(int64_t rows, int64_t d);
/* per-row ||x||_p: p = inf → max |x| (exact, NaN-propagating), p = 2 → sqrt of an fp64 sum of
 * squares rounded once to fp32 (compressors.py:332, 372; np.linalg.norm) */
int flc_quant_norm(const float* x, int64_t rows, int64_t d, int norm_p, float* norms, void* ws,
                   size_t ws_bytes, void* stream);
/* encode (compressors.py:339-365 / 376-404, the stochastic level choice); `nnz` (device, int64[rows])
 * receives the count of x != 0 per row, the quantity the reference's send-statistics count. */
int flc_quant_encode(const float* x, int64_t rows, int64_t d, int kind, int levels, int bits,
                     const float* norms, uint64_t seed, uint64_t counter, const double* compat_u,
                     uint8_t* codes, int64_t* nnz, void* ws, size_t ws_bytes, void* stream);
/* encode + decode in one pass (compressVector's round trip, compressors.py:339-365 / 376-404): the codes are
 * written exactly as flc_quant_encode writes them and out receives the value flc_quant_decode would give each code
 * (weight 1, no accumulate), computed from the code in registers instead of reading the wire back. */
int flc_quant_encode_decode(const float* x, int64_t rows, int64_t d, int kind, int levels, int bits,
                            const float* norms, uint64_t seed, uint64_t counter, const double* compat_u,
                            uint8_t* codes, int64_t* nnz, float* out, void* ws, size_t ws_bytes, void* stream);
/* philox mode, norm included: the per-row norm (as flc_quant_norm computes it, written to norms), the encode and,
 * with out != NULL, the fused decode.  p = inf with d >= 16384 and a batch of at most #CU x 32768 elements (configs[1]:
 * 10 x 417,482) runs in ONE persistent launch (one 1024-thread block per CU, a grid exchange of the per-row maxima;
 * the co-residency contract of the top-k encoders, flc_topk_status below: check flc_quant_status); otherwise two
 * launches when d >= 2048 (the encode folds the norm partials itself), three below.  The result is the same. */
int flc_quant_encode_auto(const float* x, int64_t rows, int64_t d, int kind, int levels, int bits, int norm_p,
                          uint64_t seed, uint64_t counter, uint8_t* codes, float* norms, int64_t* nnz, float* out,
                          void* ws, size_t ws_bytes, void* stream);
/* the quantizer workspace's sticky error word (4: a one-launch encode's grid exchange timed out, i.e. its blocks were
 * not all resident — the outputs of that call are invalid); copied to *err_out (device uint64), zeroed with reset */
int flc_quant_status(void* ws, uint64_t* err_out, int reset, void* stream);
/* compat mode: how many uniforms the reference draws for this batch — one per element with x != 0
 * whose y = |x| / norm is not NaN (compressors.py:339-354); norms == NULL counts x != 0 (the natural
 * compressor, compressors.py:307-316).  *count is a device int64. */
int flc_count_consumers(const float* x, int64_t rows, int64_t d, const float* norms, int64_t* count,
                        void* stream);
/* decode: v = fp32(fp32(level_value) * sign) * norm (compressors.py:357/394);
 * out = accumulate ? fmaf(row_weight, v, out) : (row_weights ? row_weight * v : v) */
int flc_quant_decode(const uint8_t* codes, int64_t rows, int64_t d, int kind, int levels, int bits,
                     const float* norms, const float* row_weights, int accumulate, float* out,
                     void* stream);

/* ------------------------------------------------------------------ natural compressor
 * (compressors.py:302-325).  Wire: one uint16 per element, 0 = zero, else sign << 15 | (e + 150)
 * for the chosen power of two 2^e, e in [-149, 127]. */
size_t flc_natural_workspace_size(int64_t n);  /* needed in compat mode only */
int flc_natural_encode(const float* x, int64_t n, uint64_t seed, uint64_t counter,
                       const double* compat_u, uint16_t* codes, int64_t* nnz, void* ws, size_t ws_bytes,
                       void* stream);
int flc_natural_decode(const uint16_t* codes, int64_t n, float weight, int accumulate, float* out,
                       void* stream);

/* ------------------------------------------------------------------ top-k sparsifier
 * (compressors.py:293-296): keeps the k largest *signed* values (NaN largest, -0 == +0); among values
 * equal to the k-th largest the highest indices are kept (the order of a stable ascending argsort).
 * Output: idx[k] ascending, val[k] the kept values bit-for-bit.  Requires 0 < k < n.
 *
 * Co-residency: the top-k and stacked encoders are ONE persistent launch of one 1024-thread block per CU
 * whose blocks hand work to each other through flags in the workspace, so every block of the launch must
 * be resident at once.  Launches of these encoders on one device are serialised by the library (stream
 * order, or an event chain across streams; not inside a stream capture); kernels of other libraries or
 * processes that occupy CUs for long stretches can delay a block past the bounded spin, which the kernel
 * records in the workspace's sticky error word instead of hanging.  flc_topk_status reads that word:
 * 0 = every call since the last reset was exact; otherwise bits 1 (digit not found), 2 (count mismatch),
 * 4 (exchange spin timeout) mean the kept set of some call may be wrong.  Check it after calls that may
 * have shared the device (fl_sim_amd does when FLC_TOPK_CHECK=1, and the GPU tests after every test). */
/* *err_out (device uint64) = the workspace's sticky error word; reset != 0 clears it (stream-ordered) */
int flc_topk_status(void* ws, uint64_t* err_out, int reset, void* stream);
/* Test hook (host only, no device): the batched encoders' pinned table ring (a ring of 32 host slots whose reuse
 * waits for an event recorded after every 8th slot's use, or drains the device) driven by `n_ops` triples
 * (kind, slot, stream id): kind 0 stages the next slot and writes (slot, wait 0 none / 1 event / 2 drain, event slot)
 * to `out`; kind 1 marks `slot` done on stream `stream id` (> 0).  Returns the triples written, or -1. */
int flc_ring_selftest(const int32_t* ops, int n_ops, int32_t* out, int n_out);
size_t flc_topk_workspace_size(int64_t n, int64_t k);
int flc_topk_encode(const float* x, int64_t n, int64_t k, int32_t* idx, float* val, void* ws,
                    size_t ws_bytes, void* stream);
/* Tile pointers (CSR row pointers over FLC_TILE-output tiles) of an ascending index stream:
 * tiles[t] = first j with idx[j] >= t * FLC_TILE, t = 0 .. ceil(n / FLC_TILE); the encoders' *_tiled
 * variants emit them alongside the wire (so that a decoder needs no index pass), flc_tile_index forms
 * them from idx alone. */
#define FLC_TILE 1024
int flc_tile_index(const int32_t* idx, int64_t k, int64_t n, uint32_t* tiles, void* stream);
int flc_topk_encode_tiled(const float* x, int64_t n, int64_t k, int32_t* idx, float* val, uint32_t* tiles,
                          void* ws, size_t ws_bytes, void* stream);
/* dense decode of an ascending sparse stream: out[idx[j]] = scale * val[j], zeros elsewhere
 * (compressors.py:289-291, 294-295); out = weight * v, or with accumulate out = fmaf(weight, v, out)
 * over the whole vector (the fused aggregation).  Workspace: a per-tile index of the stream. */
size_t flc_sparse_decode_workspace_size(int64_t n);
int flc_sparse_decode(const int32_t* idx, const float* val, int64_t k, float scale, int64_t n,
                      float weight, int accumulate, float* out, void* ws, size_t ws_bytes, void* stream);
int flc_sparse_decode_tiled(const int32_t* idx, const float* val, int64_t k, float scale, int64_t n,
                            float weight, int accumulate, float* out, const uint32_t* tiles, void* stream);

/* ------------------------------------------------------------------ stacked top-k -> 8-bit dither
 * Top-k of x (as above), then standard dithering with s = levels (<= 127), p = inf, of the k kept
 * values: the pipeline TopK(x) followed by StandardDithering on the k-sparse result.
 * Wire: idx[k] int32 ascending, codes[k] (sign << 7 | level), norm[1] fp32. */
int flc_stacked_encode(const float* x, int64_t n, int64_t k, int levels, uint64_t seed,
                       uint64_t counter, const double* compat_u, int32_t* idx, uint8_t* codes,
                       float* norm, void* ws, size_t ws_bytes, void* stream);
int flc_stacked_encode_tiled(const float* x, int64_t n, int64_t k, int levels, uint64_t seed,
                             uint64_t counter, const double* compat_u, int32_t* idx, uint8_t* codes,
                             float* norm, uint32_t* tiles, void* ws, size_t ws_bytes, void* stream);
int flc_stacked_decode(const int32_t* idx, const uint8_t* codes, int64_t k, int levels,
                       const float* norm, int64_t n, float weight, int accumulate, float* out,
                       void* ws, size_t ws_bytes, void* stream);  /* ws: flc_sparse_decode_workspace_size */
int flc_stacked_decode_tiled(const int32_t* idx, const uint8_t* codes, int64_t k, int levels,
                             const float* norm, int64_t n, float weight, int accumulate, float* out,
                             const uint32_t* tiles, void* stream);

/* Packed wire: one client's stacked wire as ONE contiguous record whose layout depends on (n, k) only, so that
 * a [clients, stride] byte buffer moves as one piece (RCCL all-gather, PCIe copy).  Returns the record size
 * (a multiple of 256 B; 0 for bad arguments) and, if offsets != NULL, the byte offsets of
 * offsets[0] norm (fp32), [1] idx (int32[k]), [2] codes (u8[max(k,16)]), [3] tiles (u32[ceil(n/FLC_TILE)+1]).
 * flc_stacked_encode_tiled writes a record when given those four pointers inside it. */
size_t flc_stacked_wire_layout(int64_t n, int64_t k, int64_t* offsets);
/* Fold of many clients' wires into one vector in ONE pass over out (the server's weighted aggregation,
 * nodes.py:1165-1180 / _fedopt.py:202-208, fused with the decode):
 *   out = (accumulate ? out : +0);  for c = 0 .. n_wires-1:  out = fmaf(weights[c], decode(record slots[c]), out)
 * elementwise, in that order — bit-identical to n_wires flc_stacked_decode_tiled(weight, accumulate=1) calls on a
 * zeroed (or the given) out.  wires: records of `stride` bytes (>= flc_stacked_wire_layout(n, k), 16-B multiple),
 * record index slots[c] holds client c; slots and weights are HOST arrays.  Replaces SURVEY §8(e)'s dense reduce
 * when the records are all-gathered: every rank folds all clients in client order, so the result does not depend on
 * the number of GPUs. */
int flc_stacked_fold_wires(const void* wires, int64_t stride, const int32_t* slots, const float* weights,
                           int n_wires, int64_t n, int64_t k, int levels, int accumulate, float* out, void* stream);
/* A compressed FedOpt round's server update in ONE pass (replaces FedOptServer.update, _fedopt.py:196-240, when each
 * client message carries its delta as a packed stacked record — the codec's call site, fl_sim_amd/compressed.py):
 * over the flat concatenation of the model's tensors (element e of the records = element e - offset_t of tensor t,
 * the order FedOptClient.communicate's delta list flattens in),
 *   a = delta * beta0;  for c = 0 .. n_records-1:  a = fmaf(weights[c], decode(records[c]), a);  delta = a;
 *   then, if theta != NULL, the optimiser's step on theta (and v): avg theta = fmaf(lr, a, theta); adagrad / yogi /
 *   adam as flc_model_fold (every rounding where torch's CPU ops round).
 * Bit-identical to decoding every record densely (flc_stacked_decode_tiled) and running flc_model_fold with
 * init_mode 0 and the step.  records: HOST array of n_records device pointers to records of the
 * flc_stacked_wire_layout(n, k) layout (16-B aligned; any device memory the stream's device can read, e.g. each client's
 * own); delta / theta / v: HOST arrays of n_tensors device pointers (v only for adaptive optimisers; pinned host
 * memory mapped into the device's address space works too), sizes summing to n.  theta == NULL: the fold alone. */
int flc_fedopt_fold_records(const void* const* records, const float* weights, int n_records, int64_t n, int64_t k,
                            int levels, float* const* delta, float* const* theta, float* const* v,
                            const int64_t* sizes, int n_tensors, float beta0, int opt, double lr, double beta2,
                            double tau, void* stream);

/* ------------------------------------------------------------------ multi-GPU exchange (RCCL over xGMI)
 * For callers outside torch; one process per GPU.  RCCL is the NCCL API on ROCm, looked
 * up on first use: $FLC_RCCL_LIB if set, else an RCCL already loaded in the process (inside a torch process, torch's
 * own, whatever its soname), else librccl.so.1.  The round's exchange is either
 *   flc_rccl_reduce: sum of the ranks' fp32 partial sums to `root` (the dense round; the cross-rank summation order is
 *     RCCL's, so the result matches one device to 1e-6 * sum|w_i d_i|), or
 *   flc_rccl_allgather: every rank's block of packed wire records to every rank (recv = nranks * bytes_per_rank, rank
 *     order), then flc_stacked_fold_wires over all clients in client order (bit-identical to one device at any N).
 * flc_comm_unique_id on one rank, its flc_comm_id_bytes() bytes shipped to the others out of band, then
 * flc_comm_init on every rank (collective; `device` >= 0: the communicator's HIP device, made current for the call
 * only — the calling thread's current device is restored).  Collectives are
 * stream-ordered and asynchronous like every other call. */
size_t flc_comm_id_bytes(void);
/* Where the RCCL symbols were found on first use (loads RCCL if not yet loaded): "env" (FLC_RCCL_LIB), "global" (the
 * process's global namespace, e.g. torch's RCCL loaded RTLD_GLOBAL), "loaded" (an already-loaded librccl* object),
 * "dlopen" (librccl.so.1), or "none" (not found; every flc_comm_* / flc_rccl_* call then fails with FLC_ECOMM). */
const char* flc_comm_rccl_origin(void);
int flc_comm_unique_id(void* id_out);
int flc_comm_init(const void* id, int nranks, int rank, int device, void** comm_out);
int flc_comm_size(void* comm, int* nranks, int* rank);
int flc_comm_destroy(void* comm);
int flc_rccl_reduce(const float* send, float* recv, int64_t n, int root, void* comm, void* stream);
int flc_rccl_allreduce(const float* send, float* recv, int64_t n, void* comm, void* stream);
int flc_rccl_allgather(const void* send, void* recv, int64_t bytes_per_rank, void* comm, void* stream);

/* ------------------------------------------------------------------ adaptive random compressor
 * (compressors.py:297-301): ind = np.random.choice(np.arange(n), size=1, p=|x| / sum|x|); out = 0,
 * out[ind] = x[ind].  Bit-exact with numpy: S in numpy's order (8192-element buffers folded in order, each
 * by pairwise_sum), p = fp32(|x| / S), the strictly sequential fp64 cumsum, cdf / cdf[-1] and
 * searchsorted(u, side='right').  Two calls, because numpy validates p before it draws u:
 *   flc_adaptive_prepare writes the check to *status (device int32): 0 ok, 1 "probabilities contain NaN",
 *     2 "probabilities do not sum to 1" (|sum p - 1| > 3.4526698e-4);
 *   flc_adaptive_select (same stream, same x and workspace) takes u in [0, 1) (compat mode: the legacy
 *     np.random.random_sample() draw, see flc_mt_random_doubles) and writes out and *index (device int64);
 *     it writes nothing when the status is non-zero.  x must be 16-byte aligned; 0 < n < 2^31. */
size_t flc_adaptive_workspace_size(int64_t n);
int flc_adaptive_prepare(const float* x, int64_t n, int32_t* status, void* ws, size_t ws_bytes, void* stream);
int flc_adaptive_select(const float* x, int64_t n, double u, int64_t* index, float* out, void* ws, size_t ws_bytes,
                        void* stream);
/* the same on a float64 x (the reference keeps it float64): S an fp64 sum of the same buffers and trees, p = |x| / S
 * in fp64, the tolerance sqrt(eps64) = 1.4901161e-8; same workspace size */
int flc_adaptive_prepare_f64(const double* x, int64_t n, int32_t* status, void* ws, size_t ws_bytes, void* stream);
int flc_adaptive_select_f64(const double* x, int64_t n, double u, int64_t* index, double* out, void* ws,
                            size_t ws_bytes, void* stream);
/* the last select's walk on this workspace, as 4 device int32: special chunks (a binade crossing or near an edge),
 * special maps taken, chunks re-run sequentially, 1 if the exact sequential chain ran instead (diagnostics: the
 * result never depends on them) */
int flc_adaptive_stats(const void* ws, size_t ws_bytes, int64_t n, int32_t* stats, void* stream);

/* the stacked encoder fused with the client delta (f1): x = local - global formed in the encoder's HBM pass
 * (FedOptClient.communicate, _fedopt.py:294-297: clone + add_(alpha=-1) per parameter tensor, then the flatten the
 * codec's flat input needs, nodes.py:300-302) — the flat delta is never written.  local, global and sizes are HOST
 * arrays (of device pointers / element counts, like flc_delta_flatten); tensors must be 4-B aligned; the element
 * order is the concatenation.  The output is bit-identical to flc_stacked_encode_tiled of the flattened delta.
 * The workspace holds the encoder's plus a tensor table (copied from the host arrays, so not graph-capturable). */
size_t flc_stacked_encode_delta_workspace_size(int64_t n, int64_t k, int n_tensors);
int flc_stacked_encode_delta(const float* const* local, const float* const* global, const int64_t* sizes,
                             int n_tensors, int64_t k, int levels, uint64_t seed, uint64_t counter, int32_t* idx,
                             uint8_t* codes, float* norm, uint32_t* tiles, void* ws, size_t ws_bytes, void* stream);

/* the stacked encoder over many clients of one round in one launch (the clients a rank encodes before the fold,
 * nodes.py:706-713 / _fedopt.py:295-308 once per client): client c's packet is bit-identical to
 * flc_stacked_encode_tiled(xs[c], n, k, levels, seeds[c], counter, ...) into idx[c], codes[c], norm[c], tiles[c]
 * (tiles may be NULL: no tile pointers; the four pointers of a wire record make client c's record).  All clients
 * have the same n and k; xs, seeds, idx, codes, norm and tiles are HOST arrays of n_clients entries (device
 * pointers / seeds).  The device's CUs are split among up to #CU clients per launch (one independent select of
 * #CU / clients blocks each, its own header, no exchange across clients); more clients run in further launches on
 * the stream.  The workspace is used afresh by every call (its headers are zeroed in the stream), so it needs no
 * zeroing by the caller, but must not be shared with single-client calls.  flc_topk_status(ws) reports the errors
 * of every client's select.  The client table is copied from the host arrays into the workspace, so the call is not
 * graph-capturable (like flc_stacked_encode_delta). */
size_t flc_stacked_encode_batch_workspace_size(int64_t n, int64_t k, int n_clients);
int flc_stacked_encode_batch(const float* const* xs, int n_clients, int64_t n, int64_t k, int levels,
                             const uint64_t* seeds, uint64_t counter, int32_t* const* idx, uint8_t* const* codes,
                             float* const* norm, uint32_t* const* tiles, void* ws, size_t ws_bytes, void* stream);

/* plain top-k of many clients in one launch (compressors.py:293-296 per client): client c's (idx, val, tiles) equal
 * flc_topk_encode_tiled(xs[c], n, k, ...); arrays and workspace as in flc_stacked_encode_batch (the two share a
 * workspace size). */
size_t flc_topk_encode_batch_workspace_size(int64_t n, int64_t k, int n_clients);
int flc_topk_encode_batch(const float* const* xs, int n_clients, int64_t n, int64_t k, int32_t* const* idx,
                          float* const* val, uint32_t* const* tiles, void* ws, size_t ws_bytes, void* stream);

/* the batched encoder fused with the clients' deltas (f1 for a round's clients): client c's packet is
 * bit-identical to flc_stacked_encode_delta(local + c * n_tensors, global, sizes, ...) with seeds[c].  local is a HOST
 * array of n_clients * n_tensors device pointers, client-major (client c's tensors at [c * n_tensors, (c+1) *
 * n_tensors)); global (n_tensors, shared by every client: the round's global model) and sizes are HOST arrays as in
 * flc_stacked_encode_delta; outputs, seeds and the workspace as in flc_stacked_encode_batch. */
size_t flc_stacked_encode_delta_batch_workspace_size(int64_t n, int64_t k, int n_clients, int n_tensors);
int flc_stacked_encode_delta_batch(const float* const* local, const float* const* global, const int64_t* sizes,
                                   int n_tensors, int n_clients, int64_t k, int levels, const uint64_t* seeds,
                                   uint64_t counter, int32_t* const* idx, uint8_t* const* codes, float* const* norm,
                                   uint32_t* const* tiles, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ other compressors
 * identical (compressors.py:273-275): out = +x;  lazy (276-283): out = x / p (fp32 division);
 * rand-k (284-292): out = 0, out[idx[j]] = scale * x[idx[j]] (idx in any order, unique). */
int flc_copy(const float* x, int64_t n, float* out, void* stream);
int flc_scale_div(const float* x, int64_t n, float p, float* out, void* stream);
int flc_randk_apply(const float* x, int64_t n, const int32_t* idx, int64_t k, float scale, float* out,
                    void* stream);
/* rand-k index set in philox mode (no host round trip): keys[e] = the Philox word of element e >> 2, as a positive
 * fp32 bit pattern; the K largest keys (flc_topk_encode_tiled on keys) are a uniformly random K-subset, ascending.
 * keys must be 16-B aligned. */
int flc_randk_keys(int64_t n, uint64_t seed, uint64_t counter, float* keys, void* stream);

/* ------------------------------------------------------------------ float64 inputs (f64.hip)
 * The reference runs every compressor on whatever dtype x has (compressors.py:267-410): on a float64 vector
 * ``np.zeros_like(x)``, ``x / P``, ``D / K * x[i]``, ``math.log2(abs(x[i]))``, ``np.linalg.norm(x, p)`` and the level
 * arithmetic all stay float64.  These are the float64 forms of the entry points above (a fp64 vector in, a fp64
 * vector out; buffers 16-B aligned).  Uniforms as for float32: compat_u = one double per consumer in index order
 * (the reference's random.random() calls; count them with flc_count_consumers_f64), or Philox (compat_u == NULL).
 *   flc_copy_f64 / flc_scale_div_f64 / flc_randk_apply_f64   IDENTICAL, LAZY (x / p), RANDK (scale * x[idx[j]])
 *   flc_natural_f64        natural compression (compressors.py:302-318): codes (uint16 per element: 0 zero,
 *                          0x7fff NaN, else sign << 15 | (e + 1075)) and / or the decoded vector; either may be NULL
 *   flc_quant_norm_f64     p = inf: max |x|; p = 2: sqrt of an fp64 sum of squares (fixed order)
 *   flc_quant_f64          standard / natural dithering (compressors.py:339-357, 376-393) with the given norm:
 *                          8-bit codes (sign << 7 | level) and / or the decoded vector lv * sign * norm; nnz =
 *                          count(x != 0) when non-NULL
 *   flc_topk_dense_f64     out = x on the K largest (ties: the highest indices), +0 elsewhere (293-296), 0 < k < n
 * Workspace: flc_f64_workspace_size(n, k) bytes (compat mode, the norm and top-k with that k; not needed by the
 * element-wise forms or by the Philox-mode encoders). */
int flc_copy_f64(const double* x, int64_t n, double* out, void* stream);
int flc_scale_div_f64(const double* x, int64_t n, double p, double* out, void* stream);
int flc_randk_apply_f64(const double* x, int64_t n, const int32_t* idx, int64_t k, double scale, double* out,
                        void* stream);
size_t flc_f64_workspace_size(int64_t n, int64_t k);  /* k: flc_topk_dense_f64's k, else 0 */
int flc_count_consumers_f64(const double* x, int64_t n, const double* norm, int64_t* count, void* ws, size_t ws_bytes,
                            void* stream);
int flc_natural_f64(const double* x, int64_t n, uint64_t seed, uint64_t counter, const double* compat_u,
                    uint16_t* codes, double* out, void* ws, size_t ws_bytes, void* stream);
int flc_natural_decode_f64(const uint16_t* codes, int64_t n, double* out, void* stream);
int flc_quant_norm_f64(const double* x, int64_t n, int norm_p, double* norm, void* ws, size_t ws_bytes, void* stream);
int flc_quant_f64(const double* x, int64_t n, int kind, int levels, const double* norm, uint64_t seed,
                  uint64_t counter, const double* compat_u, uint8_t* codes, double* out, int64_t* nnz, void* ws,
                  size_t ws_bytes, void* stream);
int flc_quant_decode_f64(const uint8_t* codes, int64_t n, int kind, int levels, const double* norm, double* out,
                         void* stream);
int flc_topk_dense_f64(const double* x, int64_t n, int64_t k, double* out, void* ws, size_t ws_bytes, void* stream);
/* the float64 workspace's sticky error word (4: flc_topk_dense_f64's grid-synchronised select timed out at a barrier,
 * i.e. its blocks were not all resident — the output of that call is invalid), as flc_topk_status reports the float32
 * encoders'; copied to *err_out (device uint64), zeroed with reset */
int flc_f64_status(void* ws, uint64_t* err_out, int reset, void* stream);

/* ------------------------------------------------------------------ client delta
 * FedOptClient.communicate (_fedopt.py:294-297): delta_t = clone(local_t) then add_(global_t, alpha=-1), i.e.
 * local_t - global_t per element, for each parameter tensor t; plus the flatten the codec's flat input needs.
 * out[off_t + i] = local[t][i] - global[t][i], off_t = sizes[0] + ... + sizes[t-1].  local, global and sizes are
 * HOST arrays (of device pointers / element counts); empty tensors are allowed. */
int flc_delta_flatten(const float* const* local, const float* const* global, const int64_t* sizes, int n_tensors,
                      float* out, void* stream);
/* the number of nonzero deltas local - global (as flc_delta_flatten forms them; NaN counts) at the k flat indices idx
 * of the concatenation — the count a standard-dithering stage's send statistics take from its input (compressors.py
 * 339-365: one entry per nonzero element) when the delta itself is never formed (flc_stacked_encode_delta).  count: one
 * device int64, written stream-ordered. */
int flc_delta_count_nonzero_at(const float* const* local, const float* const* global, const int64_t* sizes,
                               int n_tensors, const int32_t* idx, int64_t k, int64_t* count, void* stream);
/* the same count (compressors.py:339-365, one send entry per nonzero dithering input) for many clients whose deltas
 * are already flat — a round's deferred compressed messages: counts[c] = the number of nonzero xs[c][idx[c][j]], j < k
 * (NaN counts), every x of n elements, every idx of k in-range indices (a stacked record's kept indices).  xs, idx
 * and counts are HOST arrays of device pointers; each count one device int64, written stream-ordered. */
int flc_count_nonzero_at_batch(const float* const* xs, const int32_t* const* idx, int n_clients, int64_t n,
                               int64_t k, int64_t* const* counts, void* stream);

/* ------------------------------------------------------------------ aggregation
 * weighted sum of client tensors into dst, in message order, one fmaf per message per element:
 *   init_mode 0: dst = dst * beta   (avg_parameters' inertia, nodes.py:1158-1159;
 *                                   FedOptServer.update's betas[0], _fedopt.py:203)
 *   init_mode 1: dst = 0            (update_gradients, nodes.py:1173-1174)
 *   init_mode 2: dst unchanged      (add_parameters, nodes.py:1131-1132)
 *   then for m in 0..n_src-1: dst = fmaf(weights[m], srcs[m][i], dst)   (nodes.py:1132, 1178; _fedopt.py:204-208)
 * srcs and weights are HOST arrays of device pointers / fp32 weights (n_src >= 0). */
int flc_weighted_sum(const float* const* srcs, const float* weights, int n_src, int64_t n, int init_mode,
                     float beta, float* dst, void* stream);
/* a whole model in ONE launch (a model is many small tensors; two launches per tensor are launch-bound): for each
 * tensor t, dst[t] = init(dst[t]) then fmaf(weights[m], srcs[m * n_tensors + t], .) for m in message order — exactly
 * flc_weighted_sum per tensor — and, with theta != NULL, flc_fedopt_step on (theta[t], dst[t], v[t]) with the folded
 * dst[t] as the delta: FedOptServer.update in one pass (_fedopt.py:196-265).  Host arrays of device pointers;
 * n_src <= 16 (a longer message list: flc_weighted_sum, which chains); 16 tensors per launch, more in further launches
 * (tensor order).  v may be NULL for opt = avg. */
int flc_model_fold(float* const* dst, const float* const* srcs, const float* weights, int n_src, const int64_t* sizes,
                   int n_tensors, int init_mode, float beta, float* const* theta, float* const* v, int opt, double lr,
                   double beta2, double tau, void* stream);
/* avg_parameters (nodes.py:1134-1163) and update_gradients (nodes.py:1165-1180) of one round in ONE launch — what
 * the variance-reduced servers run back to back (fedprox/_fedprox.py:163-167, fedpd/_fedpd.py:197-202,
 * proxskip/_proxskip.py:212-216, pfedmac/_pfedmac.py:158-162):
 *   params[t] = params[t] * inertia, then fmaf(w_params[m], param_srcs[m][t], .) for m in order;
 *   grads[t]  = +0, then fmaf(w_grads[m], grad_srcs[m][t], .) for m in order;
 * bit-identical to flc_model_fold(init 0, beta = inertia) of the parameters followed by flc_model_fold(init 1) of the
 * gradients.  param_srcs / grad_srcs: HOST arrays [n_src][n_tensors] of device pointers; params / grads / sizes HOST
 * arrays of n_tensors; more than 16 messages chain launches (each continuing the stored partial results). */
int flc_avg_and_gradients(float* const* params, float* const* grads, const float* const* param_srcs,
                          const float* const* grad_srcs, const float* w_params, const float* w_grads, int n_src,
                          const int64_t* sizes, int n_tensors, float inertia, void* stream);
/* FedDyn's and pFedMe's server updates on a whole model, one pass per <= 16 tensors and <= 16 messages
 * (theta = the model, aux = the per-element second state; srcs[m * n_tensors + t] = message m's tensor t):
 *   FLC_SRV_FEDDYN (feddyn/_feddyn.py:172-184): h = aux, for each message in order h = fmaf(c, fl(src - theta0), h)
 *     with c = fp32(-mu / num_clients); with `fold`, theta = the avg_parameters fold of theta0 in the same pass
 *     (init_mode 0: theta0 * inertia first, then fmaf(weights[m], src, .) in order); line 184's result is discarded
 *     by the reference, so nothing follows.  Without `fold` only h is updated (theta read-only: the chained form).
 *   FLC_SRV_PFEDME (pfedme/_pfedme.py:166-175): with `fold`, a = the avg fold of theta0 (init_mode 0, or 2 when the
 *     round has no message: avg_parameters returns early), then theta = fmaf(fp32(1 - c), theta0, fl(a * fp32(c)))
 *     with c = beta; without `fold` (no sources: the fold ran in chained flc_model_fold launches and aux holds the
 *     saved theta0) theta = fmaf(fp32(1 - c), aux, fl(theta * fp32(c))). */
enum flc_server_kind { FLC_SRV_FEDDYN = 1, FLC_SRV_PFEDME = 2 };
int flc_model_fold_server(float* const* theta, float* const* aux, const float* const* srcs, const float* weights,
                          int n_src, const int64_t* sizes, int n_tensors, int kind, int fold, int init_mode,
                          float inertia, double c, void* stream);
/* the rest of FedOptServer.update after the delta average (_fedopt.py:212-265):
 *   avg:     theta = fmaf(lr, delta, theta)
 *   adagrad: v = v + delta^2;                               theta += lr * delta / (sqrt(v) + tau)
 *   yogi:    v = v - (1-beta2) * delta^2 * sign(v - delta^2); theta += ...
 *   adam:    v = v * beta2 + (1-beta2) * delta^2;            theta += ... */
int flc_fedopt_step(float* theta, const float* delta, float* v, int64_t n, int opt, double lr, double beta2,
                    double tau, void* stream);

/* the rest of FedDRServer.update once x_tilde holds its sample-weighted fold (flc_weighted_sum, init_mode 2,
 * _feddr.py:172-180), one pass:
 *   y = fmaf(alpha, theta - y, y)                       (_feddr.py:166-170)
 *   theta = prox(cx * x_til + cy * y)                   (_feddr.py:182-190; cx = coeff/eta, cy = 1/(N+1) in fp32)
 *   prox: NONE (NullRegularizer); L1: sign(t) * max(|t| - prox_c, 0) (L1Norm); SCALE: t * prox_c (L2NormSquared,
 *   prox_c = 1/(1+2 coeff); L2Norm: NONE, then the host scales by max(0, 1 - 1/||theta||) with flc_weighted_sum). */
int flc_feddr_combine(float* theta, float* y, const float* x_til, int64_t n, float alpha, float cx, float cy,
                      int prox, float prox_c, void* stream);
/* the same three on float64 models and messages (the reference's torch ops keep them float64: add_ with alpha is one
 * fp64 fma per element, the scalars stay Python doubles, sqrt is IEEE): weights, beta, lr, beta2, tau, alpha, cx, cy
 * and prox_c are used as given */
int flc_weighted_sum_f64(const double* const* srcs, const double* weights, int n_src, int64_t n, int init_mode,
                         double beta, double* dst, void* stream);
int flc_fedopt_step_f64(double* theta, const double* delta, double* v, int64_t n, int opt, double lr, double beta2,
                        double tau, void* stream);
int flc_feddr_combine_f64(double* theta, double* y, const double* x_til, int64_t n, double alpha, double cx, double cy,
                          int prox, double prox_c, void* stream);

/* ------------------------------------------------------------------ measurement
 * Record HIP events around every launch of the kernel named `kernel_name` (NULL disables);
 * flc_probe_read synchronises those events and returns the summed duration and launch count, then
 * clears the record. Used by bench.py for the live roofline figure. */
int flc_probe_set(const char* kernel_name);
int flc_probe_read(double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* FLCODEC_H_ */

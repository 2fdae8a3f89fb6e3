/*
 * fsagg.h — C ABI of libfsagg.so, the MI355X (gfx950) server-side aggregation
 * engine that backs federatedscope_amd's Aggregator.aggregate() drop-ins.
 *
 * The reference has no native code: every entry point below
 * replaces a Python/ATen loop inside federatedscope/core/aggregators.  The
 * reference interface each one stands in for is cited per function.  The
 * Python side binds these with ctypes (federatedscope_amd/_lib.py); the
 * binding stub a FederatedScope maintainer would add is in INTEGRATION.md.
 *
 * Conventions
 *  - Every pointer argument marked (device) is HBM memory owned by the caller
 *    (torch tensors' data_ptr()); the library never allocates or frees.
 *  - A "row table" is a DEVICE array of n pointers, row i being client i's
 *    flattened fp32 update of `numel` elements (the client's parameter
 *    bucket).  Order in the table = reduction order = the reference's
 *    client_feedback list order.  Rows and `out` must be 16-byte aligned.
 *  - All calls are asynchronous on `stream` (a hipStream_t; NULL = the null
 *    stream).  Return 0 on success, a negative code on failure; the message
 *    is in fsagg_last_error() (thread-local).  No C++ exception crosses the
 *    ABI.
 *  - No FMA contraction anywhere on a bit-exact path: x*w and acc+t are each
 *    rounded to fp32, exactly as ATen's CPU kernels do.
 */
#ifndef FSAGG_H_
#define FSAGG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *fsagg_stream_t; /* hipStream_t */

#define FSAGG_VERSION 2

enum fsagg_status {
  FSAGG_OK = 0,
  FSAGG_EINVAL = -1,   /* bad argument (null pointer, n < 1, misaligned) */
  FSAGG_EHIP = -2,     /* a HIP runtime call failed */
  FSAGG_ESPACE = -3,   /* workspace too small */
};

/* Element types of a client bucket (fsagg_weighted_sum_typed). */
enum fsagg_dtype {
  FSAGG_F32 = 0,
  FSAGG_F16 = 1,
  FSAGG_BF16 = 2,
  FSAGG_F64 = 3,
  FSAGG_I64 = 4, /* int64 input, fp32 output (ATen promotion of int*float) */
};

int fsagg_version(void);
const char *fsagg_last_error(void);

/*
 * Weighted sum over clients, per element, in row-table order:
 *     t_i  = fl32(x_i[p] * s_i)            (only if prescale != NULL)
 *     acc  = fl32(t_0 * w_0)
 *     acc  = fl32(acc + fl32(t_i * w_i))   for i = 1 .. n-1
 *     out[p] = base ? fl32(base[p] + acc) : acc
 * Replaces ClientsAvgAggregator._para_weighted_avg
 *   (federatedscope/core/aggregators/clients_avg_aggregator.py:60-100),
 * AsynClientsAvgAggregator._para_weighted_avg + init add
 *   (asyn_clients_avg_aggregator.py:36-40,53-84),
 * the multi-Krum average (krum_aggregator.py:35-39,79-90) and the scaled
 * average of NormboundingAggregator (normbounding_aggregator.py:35-47).
 *   rows     (device) n row pointers; weights (device) n fp32 (already
 *            rounded from the reference's double weights);
 *   prescale (device) n fp32 or NULL; base (device) numel fp32 or NULL.
 */
int fsagg_weighted_sum_f32(const float *const *rows, const float *weights,
                           const float *prescale, int n, int64_t numel,
                           const float *base, float *out,
                           fsagg_stream_t stream);

/*
 * Same contract for non-fp32 buckets (A5's dtype rules): the product x*w is
 * computed in float (f16/bf16/i64) or double (f64) and rounded to the output
 * type, then accumulated with one rounding per add.  weights are DOUBLE on
 * the device (the f64 path uses them unrounded).  out_dtype is in_dtype,
 * except FSAGG_I64 whose output is FSAGG_F32.
 */
int fsagg_weighted_sum_typed(const void *const *rows, int in_dtype,
                             const double *weights, int n, int64_t numel,
                             void *out, fsagg_stream_t stream);

/*
 * Online running mean, one client:  m = fl(fl(fl(c*m) + fl(s*x)) / d)
 * with c = cnt, s = sample_size, d = cnt + s given as fp32.
 * Replaces OnlineClientsAvgAggregator.inc (clients_avg_aggregator.py:125-142).
 */
int fsagg_online_inc_f32(float *m, const float *x, float cnt, float s,
                         float denom, int64_t numel, fsagg_stream_t stream);

/*
 * The same running mean for keys that are not float32 on both sides, with
 * ATen's dtype rules (clients_avg_aggregator.py:136-139 on any tensors):
 * a = cnt*m in m's type, b = s*x in x's type, c = a + b in common_dtype
 * (torch.promote_types of the two), out = c / (cnt + s) in common_dtype —
 * float32 when common_dtype is FSAGG_I64 (true division).  Reduced floats
 * are computed in float and rounded once per op.  out may alias m when
 * their types agree.
 */
int fsagg_online_inc_typed(const void *m, int m_dtype, const void *x,
                           int x_dtype, void *out, int common_dtype,
                           int64_t cnt, int64_t s, int64_t numel,
                           fsagg_stream_t stream);

/* out = a + b elementwise (the robust rules' init + update; e.g.
 * median_aggregator.py:37-41).  out may alias a or b. */
int fsagg_add_f32(const float *a, const float *b, float *out, int64_t numel,
                  fsagg_stream_t stream);

/*
 * Coordinate-wise median over the n rows:  (lo - (-hi)) / 2  with lo/hi the
 * lower/upper middle order statistics (== (median(T) - median(-T))/2 of
 * median_aggregator.py:43-52, bit-exact), NaN if the column holds a NaN;
 * out = base ? base + med : med.
 */
int fsagg_coord_median_f32(const float *const *rows, int n, int64_t numel,
                           const float *base, float *out,
                           fsagg_stream_t stream);

/*
 * Coordinate-wise trimmed mean: drop the k largest and k smallest of each
 * column, sum the rest, divide by `divisor` (n - 2k for trimmed mean,
 * gamma for Bulyan); out = base ? base + r : r.
 * Replaces TrimmedmeanAggregator._aggre_with_trimmedmean
 * (trimmedmean_aggregator.py:44-57) and Bulyan's second stage
 * (bulyan_aggregator.py:92-105).  Requires 2k < n.
 */
int fsagg_trimmed_mean_f32(const float *const *rows, int n, int64_t numel,
                           int k, float divisor, const float *base,
                           float *out, fsagg_stream_t stream);

/*
 * Krum pairwise distances, per key segment.  seg_off (device, int64,
 * nseg+1 entries, seg_off[0] = 0, seg_off[nseg] = numel) splits each row into
 * the state_dict keys.  Produces D (device, n*n fp32, row-major):
 *     D[a][b] = Σ_seg fl32( sqrt( Σ_{p in seg} (x_a[p] - x_b[p])^2 ) ),
 *     D[a][a] = +inf
 * — the sum over keys of per-key L2 distances of
 * KrumAggregator._calculate_distance (krum_aggregator.py:41-56) filled as in
 * _calculate_score (:58-73).  Per-key sums accumulate in fp32 within a chunk
 * and in fp64 across chunks (fixed order, deterministic).  2 <= n <= 4096
 * (FSAGG_EINVAL beyond).
 * Workspace: fsagg_pairdist_workspace_bytes(n, numel, nseg) bytes (device).
 */
size_t fsagg_pairdist_workspace_bytes(int n, int64_t numel, int nseg);
/* Coordinates per chunk of the distance kernels for (n, numel, nseg): each
 * fp32 per-chunk partial of a pair sums at most this many squared
 * differences plus its k-slice sums (<= 256), so its relative rounding
 * error is below (chunk + 256)·2^-24 (all terms are non-negative). */
int64_t fsagg_pairdist_chunk_elems(int n, int64_t numel, int nseg);
int fsagg_pairdist_f32(const float *const *rows, int n, int64_t numel,
                       const int64_t *seg_off, int nseg, float *D,
                       void *workspace, size_t workspace_bytes,
                       fsagg_stream_t stream);

/*
 * The two halves of fsagg_pairdist_f32, for the multi-GPU (parameter-range
 * sharded) Krum: every rank computes per-key squared distances over its own
 * coordinate range, the [nseg][n][n] fp64 partials are summed across ranks
 * (one RCCL all-reduce — the path's only exchange step), and every rank
 * finishes D from the summed partials.
 *   segsq (device) nseg*n*n doubles: Σ_{p in seg} (x_a[p]-x_b[p])^2, diag 0.
 *   Workspace: fsagg_pairdist_workspace_bytes(n, numel, nseg).
 */
int fsagg_pairdist_segsq_f32(const float *const *rows, int n, int64_t numel,
                             const int64_t *seg_off, int nseg, double *segsq,
                             void *workspace, size_t workspace_bytes,
                             fsagg_stream_t stream);
int fsagg_pairdist_finish_f64(const double *segsq, int n, int nseg, float *D,
                              fsagg_stream_t stream);

/*
 * Per-row squared L2 norm in fp64 (deterministic two-level reduction):
 * sq[i] = Σ_p x_i[p]^2.  The norm of NormboundingAggregator's flattened update
 * (normbounding_aggregator.py:39-41, torch.norm(param, p=2)).
 * Workspace: fsagg_rownorm_workspace_bytes(n, numel).
 */
size_t fsagg_rownorm_workspace_bytes(int n, int64_t numel);
int fsagg_row_sqnorm_f32(const float *const *rows, int n, int64_t numel,
                         double *sq, void *workspace, size_t workspace_bytes,
                         fsagg_stream_t stream);

/*
 * FedOpt server step on the aggregated bucket (fedopt_aggregator.py:26-44,
 * optimizer built by name, core/auxiliaries/optimizer_builder.py:53-56):
 * per element g = param - avg (negated with FSAGG_OPT_MAXIMIZE), then one
 * torch.optim single-tensor step in place on param and the optimizer state
 * buckets:
 *   SGD      state0 = momentum buffer;
 *   Adam     state0 = exp_avg, state1 = exp_avg_sq, state2 = max_exp_avg_sq
 *            (amsgrad); AdamW = Adam with FSAGG_OPT_DECOUPLED: param is
 *            first scaled by decay_mul = 1 - lr·weight_decay;
 *   Adagrad  state0 = state_sum; clr = lr / (1 + (step - 1)·lr_decay);
 *   RMSprop  state0 = square_avg, state1 = momentum buffer (momentum > 0),
 *            state2 = grad_avg (FSAGG_OPT_CENTERED); alpha the smoothing
 *            constant.
 * Scalars are the host's doubles; the kernels convert them to the
 * parameter type as ATen does (Adam's step_size = lr / (1 - beta1^t) and
 * bias_correction2_sqrt = (1 - beta2^t)^0.5 are computed on the host, as
 * torch does).  Tolerance-pinned: ATen's CPU optimizer arithmetic (fmadd
 * in the vectorised body) is ISA-dependent.  _f32 for float32 parameters,
 * _f64 for float64 ones.
 */
enum fsagg_opt_kind { FSAGG_OPT_SGD = 0, FSAGG_OPT_ADAM = 1,
                      FSAGG_OPT_ADAGRAD = 2, FSAGG_OPT_RMSPROP = 3 };
enum fsagg_opt_flags { FSAGG_OPT_NESTEROV = 1, FSAGG_OPT_FIRST_STEP = 2,
                       FSAGG_OPT_AMSGRAD = 4, FSAGG_OPT_DECOUPLED = 8,
                       FSAGG_OPT_MAXIMIZE = 16, FSAGG_OPT_CENTERED = 32 };
typedef struct fsagg_opt_params {
  int kind;
  int flags;
  double lr, momentum, dampening, weight_decay;
  double beta1, beta2, eps, step_size, bias_correction2_sqrt;
  double alpha;      /* RMSprop smoothing constant */
  double clr;        /* Adagrad's decayed learning rate for this step */
  double decay_mul;  /* AdamW: 1 - lr * weight_decay */
} fsagg_opt_params;
int fsagg_server_opt_step_f32(float *param, const float *avg, float *state0,
                              float *state1, float *state2, int64_t numel,
                              const fsagg_opt_params *hp,
                              fsagg_stream_t stream);
int fsagg_server_opt_step_f64(double *param, const double *avg,
                              double *state0, double *state1, double *state2,
                              int64_t numel, const fsagg_opt_params *hp,
                              fsagg_stream_t stream);

/*
 * Quantised / packed upload → fp32 client-stack row, in one launch.
 * `src` (device) holds one client's packed wire bytes; `segs` (device) is an
 * array of nseg records (32 B each, naturally aligned):
 *     struct { int64_t src_byte_off, dst_elem_off, len;
 *              int32_t kind, scale_idx; }
 * kind FSAGG_WIRE_I8 / _I16: out[dst + i] = fl32(float(q[i]) * scales[idx])
 *   — the server's symmetric_uniform_dequantization `value * alpha`
 *   (federatedscope/core/compression/utils.py:70-90; int8/int16 codes times
 *   the fp32 scale tensor, one fp32 rounding), fused with the H2D scatter;
 * kind FSAGG_WIRE_F32: out[dst + i] = src_f32[i] (unquantised keys).
 * scales (device) holds the upload's nscale per-key fp32 scales; max_len
 * is the longest segment.  src_bytes / out_len are the extents of the
 * packed input and of the fp32 row: the segment table lives on the device,
 * so each segment is checked there, and one that does not fit both (or
 * names an unknown kind / scale) is skipped — it writes nothing.  Replaces Server.callback_funcs_model_para's
 * dequantisation step (federatedscope/core/workers/server.py:946-960).
 */
enum fsagg_wire_kind { FSAGG_WIRE_F32 = 0, FSAGG_WIRE_I8 = 1,
                       FSAGG_WIRE_I16 = 2, FSAGG_WIRE_B64_F32 = 3,
                       FSAGG_WIRE_ZERO = 4 };
int fsagg_wire_unpack_f32(const void *src, int64_t src_bytes,
                          const void *segs, const float *scales, int nscale,
                          int nseg, int64_t max_len, float *out,
                          int64_t out_len, fsagg_stream_t stream);

/*
 * Base64 (gRPC) upload → fp32 client-stack row, in one launch.  Replaces
 * the host decode of every tensor the gRPC transport ships as
 * base64(pickle(tensor)) (federatedscope/core/message.py:8-9,110-124 →
 * core/auxiliaries/utils.py:95-105 param2tensor, called per key by
 * clients_avg_aggregator.py:86-87); the host parses only the pickle framing.
 * `text` (device, 4-byte aligned, text_bytes a multiple of 4) holds base64
 * characters; `segs` (device) the same 32-B records as above, with
 *   kind FSAGG_WIRE_B64_F32: out[dst + i] = the fp32 whose 4 bytes are
 *       decoded bytes src + 4i .. src + 4i + 3 of `text` (src counts
 *       DECODED bytes: decoded byte b comes from the 4-char group at
 *       text + 4*(b/3)); bit-exact little-endian reinterpretation;
 *   kind FSAGG_WIRE_ZERO: out[dst + i] = 0 (padding, absent keys);
 *   scale_idx is unused (-1).  max_len is the longest segment (elements).
 * A segment outside the decoded extent or the row writes nothing and sets
 * *status = 2; a non-alphabet character ('=' included) in a decoded group
 * sets *status = 1 (`status`: a device word the caller zeroes and reads).
 */
int fsagg_b64_unpack_f32(const void *text, int64_t text_bytes,
                         const void *segs, int nseg, int64_t max_len,
                         float *out, int64_t out_len, uint32_t *status,
                         fsagg_stream_t stream);

/*
 * Secret-sharing FedAvg (cfg.federate.use_ss) in one pass:
 *     acc = Σ_i double(x_i[p]) * w  (list order; w = 1.0, or 1/n when
 *                                    ignore_weight is also set — the
 *                                    reference tests it first, :77-82;
 *                                    int64 shares converted round-to-
 *                                    nearest, as numpy)
 *     if recover:  x = acc mod `mod` (numpy float remainder)
 *                  r = x > maximum ? -(mod - x) / epsilon : x / epsilon
 *                  out[p] = fl32(r / total)
 *     else:        out_sum[p] = acc
 * Replaces the use_ss branch of ClientsAvgAggregator._para_weighted_avg
 * (clients_avg_aggregator.py:79-98) with AdditiveSecretSharing.
 * fixedpoint2float (federatedscope/core/secret_sharing/secret_sharing.py:
 * 88-98) as recover_fun.  rows (device) n pointers to float64 or int64
 * shares (row_is_int, device, n bytes); mod/maximum/epsilon are the
 * AdditiveSecretSharing constants as doubles (mod = float(2*2^size + 1)).
 * Every share row must be 16-byte aligned.
 */
int fsagg_ss_recover_f32(const void *const *rows, const uint8_t *row_is_int,
                         int n, int64_t numel, double weight, double mod,
                         double maximum, double epsilon, double total,
                         int recover, float *out, double *out_sum,
                         fsagg_stream_t stream);

/*
 * Per-row, per-key squared L2 distance to a base row, in fp64:
 *     sq[i][s] = Σ_{p in seg s} fl32(x_i[p] - base[p])^2   (base may be NULL)
 * The ‖local − last‖² terms of calc_l2_dissim / calc_blocal_dissim
 * (federatedscope/core/monitors/metric_calculator.py:309-372).
 * seg_off (device) nseg+1 int64 offsets as for fsagg_pairdist_f32.
 * Workspace: fsagg_delta_sqnorm_workspace_bytes(n, numel, nseg).
 */
size_t fsagg_delta_sqnorm_workspace_bytes(int n, int64_t numel, int nseg);
int fsagg_delta_sqnorm_f32(const float *const *rows, int n, int64_t numel,
                           const float *base, const int64_t *seg_off,
                           int nseg, double *sq, void *workspace,
                           size_t workspace_bytes, fsagg_stream_t stream);

/*
 * Weighted sum of client deltas, per element in row-table order from +0:
 *     out[p] = Σ_i fl32(w_i * fl32(x_i[p] - base[p]))
 * The global update Σ_i w_i (local_i − last) of calc_blocal_dissim
 * (federatedscope/core/monitors/metric_calculator.py:342-349;
 * `global_grads[k] += weights[i] * v` with fp32 tensors).  weights (device)
 * n fp32 (the host's doubles rounded, as ATen casts the scalar).
 */
int fsagg_delta_wsum_f32(const float *const *rows, const float *weights,
                         int n, int64_t numel, const float *base, float *out,
                         fsagg_stream_t stream);

/*
 * Key-table forms of the two metric passes, for client dicts that are
 * already device-resident (no staging copy): keys (device) is an n x nseg
 * row-major table whose entry [i][s] points at client i's fp32 tensor for
 * key s (seg_off[s+1] - seg_off[s] elements, any 4-byte alignment);
 * base_keys (device) nseg pointers to the base model's tensors (may be NULL
 * for the sqnorm).  numel = seg_off[nseg].  Results are bit-identical to the
 * flat forms over the concatenated rows; the wsum's out stays flat.
 * Reference: the same metric_calculator.py:309-372 loops, which index the
 * clients' state dicts key by key.
 */
int fsagg_delta_sqnorm_keys_f32(const float *const *keys, int n,
                                int64_t numel, const float *const *base_keys,
                                const int64_t *seg_off, int nseg, double *sq,
                                void *workspace, size_t workspace_bytes,
                                fsagg_stream_t stream);
int fsagg_delta_wsum_keys_f32(const float *const *keys, const float *weights,
                              int n, int64_t numel,
                              const float *const *base_keys,
                              const int64_t *seg_off, int nseg, float *out,
                              fsagg_stream_t stream);

/*
 * calc_blocal_dissim's two client passes in one read of the clients: sq as
 * fsagg_delta_sqnorm_f32 (per-row, per-key Σ fl32(x − base)² in fp64; a
 * different fp64 summation order, so within ~1e-15 relative of it, not
 * bit-identical) and out as fsagg_delta_wsum_f32 (bit-identical).  base is
 * required.  The _keys form takes the key tables of the two key-table
 * passes above.  Workspace: fsagg_delta_sqnorm_wsum_workspace_bytes.
 * Reference: metric_calculator.py:309-357 (one loop over the clients'
 * `local − last` for the norms, another for the global update).
 */
size_t fsagg_delta_sqnorm_wsum_workspace_bytes(int n, int64_t numel,
                                               int nseg);
int fsagg_delta_sqnorm_wsum_f32(const float *const *rows,
                                const float *weights, int n, int64_t numel,
                                const float *base, const int64_t *seg_off,
                                int nseg, double *sq, float *out,
                                void *workspace, size_t workspace_bytes,
                                fsagg_stream_t stream);
int fsagg_delta_sqnorm_wsum_keys_f32(const float *const *keys,
                                     const float *weights, int n,
                                     int64_t numel,
                                     const float *const *base_keys,
                                     const int64_t *seg_off, int nseg,
                                     double *sq, float *out, void *workspace,
                                     size_t workspace_bytes,
                                     fsagg_stream_t stream);

/*
 * Stage device-resident client updates into the client stack in ONE launch
 * (the per-key copies of ClientStack.load for GPU-resident state_dicts;
 * federatedscope/core/workers/server.py:966-970 stores the dicts that the
 * aggregators then read key by key).  src (device) is an n x nseg row-major
 * table of fp32 key tensors (NULL: the client lacks that key, its row keeps
 * its contents); dst_rows (device) n row pointers; key_off / key_len (device)
 * nseg int64 offsets into a row and lengths; the bucket is listed as nchunk
 * chunks (chunk_key int32, chunk_start int64, device) of at most
 * FSAGG_STACK_CHUNK coordinates that never straddle a key.  n <= 65535.
 */
#define FSAGG_STACK_CHUNK 2048
int fsagg_gather_rows_f32(const float *const *src, int n, int nseg,
                          float *const *dst_rows, const int64_t *key_off,
                          const int64_t *key_len, const int32_t *chunk_key,
                          const int64_t *chunk_start, int nchunk,
                          fsagg_stream_t stream);

/*
 * ---- Client rows read in place ("row sets") ------------------------------
 * The reference's aggregators index every client's state_dict key by key
 * (clients_avg_aggregator.py:70-91, median_aggregator.py:45-48,
 * krum_aggregator.py:48-53); when the uploads are already device tensors
 * (the reference's multi-GPU mode receives them on cuda:0,
 * core/parallel/parallel_runner.py:282-293), the kernels below read them
 * where they lie — no staging copy into a stack.
 *
 * A row set addresses client i's value of bucket coordinate p, p inside key
 * segment s, at  tab[s*ss + i][p]  — each entry is a "virtual base":
 * the key tensor's pointer minus 4 * (the key's bucket offset).  A stacked
 * slab is the special case ss = 0 (every segment of client i starts at its
 * row), a segment-major [nseg][n] key table has ss = n (one chunk's client
 * pointers are contiguous: batched scalar loads).  A NULL entry means the
 * client lacks that key: the weighted sum skips it (the reference's
 * `if key not in local_model: continue`), the order statistics and Krum
 * require every entry.
 * The bucket is processed as a device array of chunks that never straddle
 * a key, built once per layout by the caller: chunk c covers coordinates
 * [lo, lo + len) of segment seg, len <= the call's chunk unit.
 */
typedef struct fsagg_rows {
  const float *const *tab; /* (device) row-pointer table */
  int64_t ss;              /* table stride per key segment (0 or >= n) */
  int n;                   /* clients */
  int nseg;                /* key segments */
} fsagg_rows;

typedef struct fsagg_chunk {
  int64_t lo;  /* first bucket coordinate */
  int32_t len; /* coordinates in the chunk */
  int32_t seg; /* key segment */
} fsagg_chunk;

/* Chunk unit (coordinates) the weighted-sum row-set kernel expects for a
 * bucket of `numel` coordinates (its per-lane vector width x 1024). */
int64_t fsagg_wsum_chunk_elems(int64_t numel);
/* The same for n clients: with n >= 150 the kernel takes wider chunks
 * (fewer, longer workgroups; measured faster at 200 x 6.6M). */
int64_t fsagg_wsum_chunk_elems_n(int64_t numel, int n);

/* A/B knob: the row-set kernel's chunk width V (chunk_elems = 1024·V) that
 * fsagg_wsum_chunk_elems[_n] return — 24, 16, 8, 4 or 1; 0 (or anything
 * else) = the built-in rule.  Results do not depend on it.  Returns the
 * previous setting. */
int fsagg_wsum_set_rows_width(int v);

/*
 * fsagg_weighted_sum_f32 over a row set: out[p] for every chunk coordinate,
 * clients in table order, NULL entries skipped (the first present client
 * initialises the accumulator, as client 0 does in the reference).
 * base (device) nseg' virtual base pointers with stride base_ss (0: one
 * entry for every segment), or NULL.  out is a flat bucket.  Every non-NULL
 * entry, base entry and out must be 16-byte aligned at every chunk start
 * (chunk lo multiple of 4); chunk_elems = fsagg_wsum_chunk_elems(...).
 */
int fsagg_weighted_sum_rows_f32(const fsagg_rows *rows,
                                const fsagg_chunk *chunks, int nchunk,
                                int64_t chunk_elems, const float *weights,
                                const float *prescale,
                                const float *const *base, int64_t base_ss,
                                float *out, fsagg_stream_t stream);

/* Coordinate-wise median / trimmed mean over a row set (chunk unit
 * FSAGG_ROWS_OS_CHUNK, no NULL entries); same results as the flat forms.
 * numel = the bucket extent (every chunk inside [0, numel)). */
#define FSAGG_ROWS_OS_CHUNK 256
int fsagg_coord_median_rows_f32(const fsagg_rows *rows,
                                const fsagg_chunk *chunks, int nchunk,
                                int64_t numel, const float *const *base,
                                int64_t base_ss, float *out,
                                fsagg_stream_t stream);
int fsagg_trimmed_mean_rows_f32(const fsagg_rows *rows,
                                const fsagg_chunk *chunks, int nchunk,
                                int64_t numel, int k, float divisor,
                                const float *const *base, int64_t base_ss,
                                float *out, fsagg_stream_t stream);

/* Tuning hook of the order statistics above (no reference counterpart):
 * the client count from which 64 < n <= 255 runs the two-wave select
 * kernel (each column's rows split over two waves of one workgroup) instead
 * of the one-wave kernel; both give identical medians and trimmed means
 * within the stated tolerance.  n < 0 restores the default; returns the
 * previous value.  Process-wide; for A/B measurements. */
int fsagg_orderstat_set_pair_min(int n);
/* The same for 255 < n: with n >= 0, every n in (255, n] (n <= 512) takes
 * the K-wave kernel, which reads each column once with its rows split over
 * a workgroup's waves, for both statistics; n < 0 restores the default
 * (the median for 384 <= n <= 512, where it measured faster; otherwise the
 * one-lane streaming kernel, two passes).  Returns the previous median
 * upper bound.  For tests and A/B measurements. */
int fsagg_orderstat_set_group_max(int n);
/* The K-wave kernel's client range [lo, hi] for both statistics, from 65
 * clients up (below 256 it then replaces the two-wave kernel); lo < 0
 * restores the defaults.  Returns the previous median lower bound.  And
 * its waves per workgroup, 2..8 (anything else: the default 8); returns
 * the previous count.  For tests and A/B measurements. */
int fsagg_orderstat_set_group_range(int lo, int hi);
int fsagg_orderstat_set_group_waves(int k);

/* Krum per-key squared distances over a row set: segment s covers
 * [seg_lo[s], seg_end[s]) (device int64 arrays; keys may leave gaps between
 * them, which are never read); numel = the bucket extent (for planning).
 * Output as fsagg_pairdist_segsq_f32.  Workspace:
 * fsagg_pairdist_workspace_bytes(n, numel, nseg). */
int fsagg_pairdist_rows_segsq_f32(const fsagg_rows *rows,
                                  const int64_t *seg_lo,
                                  const int64_t *seg_end, int64_t numel,
                                  double *segsq, void *workspace,
                                  size_t workspace_bytes,
                                  fsagg_stream_t stream);

/* Krum per-key squared distances on the matrix cores (n <= 256; segsq as
 * fsagg_pairdist_rows_segsq_f32).  d²(a, b) = G_aa + G_bb − 2·G_ab from a
 * Gram matrix of the rows centred on a central client (the argmin of the
 * summed distances over the first 2048 coordinates of every key), every
 * fp32 value split exactly into three bf16 limbs and the six limb products
 * of weight >= 2^-16 accumulated by v_mfma_f32_16x16x32_bf16, fp32 within
 * one k-step of 32 coordinates, fp64 beyond.  err[s][a][b] (fp64, same
 * shape as segsq): a worst-case bound on |segsq − the exact squared
 * distance of key s's fp32 rows| — the dropped limb products, the MFMA's
 * rounding of each 32-product dot, the fp64 sums, the centring and
 * underflow, each bounded through S = sqrt(G'aa) + sqrt(G'bb) (DESIGN
 * §3.3) — or +inf where d² came out negative beyond it or is not finite.
 * Sums of segsq and err over disjoint coordinate ranges (ranks) stay
 * valid.  Replaces the same torch.dist loop (krum_aggregator.py:41-73) as
 * fsagg_pairdist_f32, with fsagg_pairgram_finish_f32 in place of
 * fsagg_pairdist_finish_f64.  The rows stream through LDS in 512-B runs
 * per row (global_load_lds), whatever their placement.  Up to 112 clients
 * one workgroup per chunk forms every 16x16 tile pair; up to 128 one
 * 8-tile workgroup, up to 208 one 13-tile workgroup of 16 waves, up to 256
 * six 8-tile workgroups per chunk (tile groups of 4 paired up, each pair
 * of tiles formed once; XCD-grouped, so a chunk's rows are read from HBM
 * once and from L2 after).  Workspace:
 * fsagg_pairgram_workspace_bytes(n, numel, nseg) (0 when n is outside
 * 2..256). */
size_t fsagg_pairgram_workspace_bytes(int n, int64_t numel, int nseg);
/* Tuning hook (no reference counterpart): which workgroups form the Gram
 * passes for n > 64.  1 (default): up to 112 clients one 4-wave workgroup
 * per chunk holding every tile (the n <= 64 form, one workgroup per CU),
 * then tile-split workgroups (every tile split once per workgroup, each
 * wave forming its share of the tile pairs) — 8 tiles on 8 waves up to 128
 * clients, all 13 tiles on 16 waves above; 2: 8-tile workgroups for every
 * n > 64 (four per chunk above 128); 3: the one-workgroup form up to 128
 * clients (13 tiles above as 1); 0: projective-plane lines throughout;
 * on < 0
 * restores the default.  segsq / err agree within the stated bounds.
 * Returns the previous setting.  For A/B measurements. */
int fsagg_pairgram_set_block8(int on);
/* The current setting of fsagg_pairgram_set_block8 (keys of captured
 * launch chains, whose kernels it selects). */
int fsagg_pairgram_block8(void);
/* Every Gram workgroup-form setting above in one value (block8 | stages << 2
 * | fused << 5 | desync << 6 | chunks << 22): the key of a captured launch
 * chain, read in one call. */
int64_t fsagg_pairgram_knobs(void);
/* The chunk kernel's LDS stages (n <= 112 forms): 1 (default) compact —
 * the n client rows, three buffers where they fit (two stages in flight);
 * 0 the full-tile stages of round 5 (16·NT rows + the centre's, one in
 * flight); 2 the compact stages with early release (a stage's buffer is
 * refilled once every wave has read its fragments, so every buffer's stage
 * is in flight under the compute); 3 the compact stages with each MFMA
 * cluster at s_setprio 1; 4 the default stages with plain loads instead
 * of non-temporal ones (the full-tile forms above 64 clients too);
 * < 0 restores the default.  Returns the
 * previous setting.  For A/B measurements; the results are identical. */
int fsagg_pairgram_set_stages(int mode);
/* The main pass's target chunk count for the n <= 112 forms (default 1024,
 * two rounds of two workgroups per CU; <= 0 restores it).  Returns the
 * previous setting.  For A/B measurements: only the fp64 summation order of
 * the chunk partials changes. */
int fsagg_pairgram_set_chunks(int chunks);

/* A/B knob: delay the start of about half of the Gram main pass's
 * workgroups (bits 0-1: which — 1 odd blocks, 2 block bit 8, 3 block bit 9;
 * bits 2+: the delay in 512-cycle sleeps; 0 = off, the default).  Returns
 * the previous setting. */
int fsagg_pairgram_set_desync(int mode);
/* A/B knob: 1 (default) the fused chain tail — the centre picked by the
 * last of the sample pass's pair-sum workgroups, each key's d², bounds and
 * the finish in one launch (six launches per chain); 0 the round-5 chain of
 * eight launches; < 0 restores the default.  The results are
 * bit-identical.  Returns the previous setting. */
int fsagg_pairgram_set_fused(int on);
int fsagg_pairgram_rows_segsq_f32(const fsagg_rows *rows,
                                  const int64_t *seg_lo,
                                  const int64_t *seg_end, int64_t numel,
                                  double *segsq, double *err,
                                  void *workspace, size_t workspace_bytes,
                                  fsagg_stream_t stream);

/* Krum's n×n distance matrix from fsagg_pairgram_rows_segsq_f32's output:
 * D[a][b] = Σ_s fl32(sqrt(segsq[s][a][b])) in key order (fp32, as
 * fsagg_pairdist_finish_f64 and the reference's `distance +=
 * torch.dist(...)`, krum_aggregator.py:45-56), D[a][a] = +inf;
 * bound[a][b] (fp32, rounded up; may be NULL) a worst-case bound on
 * |Σ_s sqrt(segsq_s) − Σ_s (exact per-key distance)| — Σ_s of the worst
 * move of sqrt over [segsq_s ± err_s] — that the caller certifies its Krum
 * selection with; ill[a*n + b] = 1 where that bound exceeds tol · Σ_s d_s,
 * or d² came out negative beyond its bound, or D is not finite — the
 * caller recomputes those pairs with fsagg_pairdist_rows_segsq_f32 on the
 * clients involved (tol = +inf: only the non-finite ones).  dist64 (fp64,
 * may be NULL): Σ_s sqrt(segsq[s][a][b]) in fp64, the sum bound[a][b]
 * bounds without D's fp32 rounding (+inf on the diagonal) — what the
 * caller certifies against. */
int fsagg_pairgram_finish_f32(const double *segsq, const double *err, int n,
                              int nseg, double tol, float *D, uint32_t *ill,
                              float *bound, double *dist64,
                              fsagg_stream_t stream);

/* fsagg_pairgram_rows_segsq_f32 and fsagg_pairgram_finish_f32 in one call
 * (the unsharded path). */
int fsagg_pairgram_rows_f32(const fsagg_rows *rows, const int64_t *seg_lo,
                            const int64_t *seg_end, int64_t numel, double tol,
                            double *segsq, double *err, float *D,
                            uint32_t *ill, float *bound, double *dist64,
                            void *workspace, size_t workspace_bytes,
                            fsagg_stream_t stream);

/* Krum distances of a few selected clients to every client, in fp64 — the
 * rows of D that decide a selection the Gram path's bounds leave ambiguous
 * (the same torch.dist loop, krum_aggregator.py:41-73, for |sel| × n pairs;
 * no reference counterpart of its own).  sel (device int32 [nsel], 1 <=
 * nsel <= FSAGG_PAIRSEL_MAX_SEL, 2 <= n <= FSAGG_PAIRSEL_MAX_CLIENTS):
 * segsq[s][a][b] (device fp64 [nseg][nsel][n]) = Σ_{p in key s} (x_sel[a][p]
 * − x_b[p])² over the chunks (chunk unit FSAGG_PAIRSEL_CHUNK), fp64
 * differences, squares and sums in a fixed order (deterministic; relative
 * error below (coordinates + 64)·2^-53).  Sums over disjoint coordinate
 * ranges (ranks) stay valid.  Workspace:
 * fsagg_pairsel_workspace_bytes(nsel, n, nchunk). */
#define FSAGG_PAIRSEL_MAX_SEL 32
#define FSAGG_PAIRSEL_MAX_CLIENTS 256
#define FSAGG_PAIRSEL_CHUNK 2048
size_t fsagg_pairsel_workspace_bytes(int nsel, int n, int nchunk);
int fsagg_pairsel_rows_segsq_f64(const fsagg_rows *rows, const int *sel,
                                 int nsel, const fsagg_chunk *chunks,
                                 int nchunk, double *segsq, void *workspace,
                                 size_t workspace_bytes,
                                 fsagg_stream_t stream);
/* D[a][b] (device fp64 [nsel][n]) = Σ_s sqrt(segsq[s][a][b]) in key order,
 * +inf where b == sel[a] (krum_aggregator.py:67-69). */
int fsagg_pairsel_finish_f64(const double *segsq, const int *sel, int nsel,
                             int n, int nseg, double *D,
                             fsagg_stream_t stream);

/* Per-(client, key segment) squared L2 norms over a row set in fp64:
 * sq[i][s] = Σ_{p in s} x_i[p]^2 (0 for a NULL entry), summed in a fixed
 * order (deterministic).  The norm of NormboundingAggregator's flattened
 * update over the server keys a client holds (normbounding_aggregator.py:
 * 35-57).  Any chunk unit.  Workspace: fsagg_rows_sqnorm_workspace_bytes. */
size_t fsagg_rows_sqnorm_workspace_bytes(int n, int nchunk);
int fsagg_rows_sqnorm_f32(const fsagg_rows *rows, const fsagg_chunk *chunks,
                          int nchunk, double *sq, void *workspace,
                          size_t workspace_bytes, fsagg_stream_t stream);

/* Norm bounding's per-client scale from sq [n][nseg] (device, as
 * fsagg_rows_sqnorm_f32 writes it), on the device so the weighted sum that
 * consumes it (its `prescale`) follows without a host round trip
 * (normbounding_aggregator.py:39-40): norm = fl32(sqrt(Σ_s sq[i][s]));
 * prescale[i] = fl32(fl32(1 / norm) · bound) if norm > bound (fp32
 * compare), else 1.  ``bound`` is fl32 of the configured bound. */
int fsagg_normbound_prescale_f32(const double *sq, int n, int nseg,
                                 float bound, float *prescale,
                                 fsagg_stream_t stream);

/*
 * Peer assembly over xGMI (strong scaling across the GPUs of one node,
 * SURVEY §8(e)).  Each GPU owns a parameter range of every client, reduces
 * it and writes the result straight into every GPU's copy of the output
 * (its own and its peers', imported through IPC handles) — the gather is
 * the producing kernel's epilogue instead of a separate collective.  Stands
 * in for the reference's device-resident multi-GPU transfer of model
 * tensors (core/communication.py:61-76, core/parallel/parallel_runner.py:
 * 22-24,243-302: per-key dist.send / dist.recv between ranks).
 *
 * fsagg_peer_alloc   `bytes` of zeroed, UNCACHED device memory on `device`
 *                    (hipDeviceMallocUncached: peers' xGMI stores and local
 *                    loads meet in memory, no stale L2 line) — the one
 *                    allocation the library makes; free with
 *                    fsagg_peer_free.
 * fsagg_peer_handle  the allocation's IPC handle (fsagg_peer_handle_bytes()
 *                    bytes) for the peer processes;
 * fsagg_peer_open    a peer's handle mapped on `device` (peer access enabled
 *                    lazily); fsagg_peer_close unmaps it.
 * fsagg_peer_pci_bus_id  `device`'s PCI bus id (buf of len >= 16 bytes);
 * fsagg_peer_can_access  1 if `device` can access the GPU with that bus id
 *                    (or it is `device`), 0 if it cannot, 2 if that GPU is
 *                    not visible to this process (nothing to check), < 0 on
 *                    error.
 * fsagg_weighted_sum_bcast_f32  fsagg_weighted_sum_f32 whose result goes to
 *                    `nout` (<= FSAGG_MAX_PEERS) outputs: outs is a HOST
 *                    array of device pointers (own and peer buffers, each
 *                    16-byte aligned), every one receiving the same bits.
 * fsagg_peer_push_f32  the epilogue of the rules without a fused broadcast
 *                    (order statistics, row-set averages through
 *                    Aggregator.aggregate()): src[0, n) — this rank's
 *                    finished piece in its own copy — stored into each of
 *                    the `ndst` peer copies (dsts: a HOST array of device
 *                    pointers, all 16-byte aligned, like src).
 * fsagg_peer_barrier  after the bcast kernel, on the same stream: stores
 *                    `epoch` into every rank's flag word for `rank`
 *                    (flags[r] = rank r's array of `world` uint32, own and
 *                    imported), then waits until every rank's word in this
 *                    rank's array reached `epoch` (epochs increase by one
 *                    per call; compared modulo 2^32).  A wait longer than
 *                    `timeout_ticks` of the 100 MHz constant clock stores
 *                    1 + the missing rank into status[0] and ends instead
 *                    of hanging; on exit the barrier stores `epoch` into
 *                    status[1].  status: two device-visible words (the
 *                    mapped host block of fsagg_peer_status_alloc, which the
 *                    host reads without a copy, or device memory).
 * fsagg_peer_status_alloc  a zeroed 64-byte word block in pinned, mapped
 *                    host memory: *host for the host to read once the
 *                    barrier's stream has passed it (no device-to-host
 *                    copy), *dev for fsagg_peer_barrier's `status`; free
 *                    with fsagg_peer_status_free.
 */
#define FSAGG_MAX_PEERS 8

/* fsagg_weighted_sum_f32 / _bcast_f32 with the tables on the HOST: `rows`
 * (n device addresses, 16-byte aligned), `weights` and `prescale` (NULL:
 * none) are host arrays of n <= FSAGG_HOSTTAB_MAX_CLIENTS entries, copied
 * into the launch's kernel arguments — nothing is uploaded before the
 * launch.  `outs`: host array of `nout` (1..FSAGG_MAX_PEERS) output
 * addresses (this GPU's first, then peers' imported copies), each receiving
 * the same numel results.  Same arithmetic, bit for bit.  Replaces the
 * per-call table uploads of ClientsAvgAggregator.aggregate() on a flat row
 * set (clients_avg_aggregator.py:60-100 over fresh uploads,
 * core/parallel/parallel_runner.py:290-293). */
#define FSAGG_HOSTTAB_MAX_CLIENTS 128
/* Host plumbing for the small per-call tables (row tables, weights, chunk
 * lists; no reference counterpart): copy `nbytes` from host `src` into the
 * caller's pinned staging slot `stage` and from there, on `copy_stream`,
 * into device `dst` (slot `slot` of an `nslot`-slot device ring, nslot <=
 * 256); `consumer` waits for the copy.  The pinned slot is refilled only
 * after its previous copy ran; the device slot is overwritten only after
 * the consumer work enqueued within nslot/2 uploads of its previous use
 * (so a consumer must launch within nslot/2 uploads of its table's).  One
 * call, a few microseconds of host time (a torch-level upload costs ~33).
 * fsagg_upload_wait: `stream` waits for slot `slot`'s copy. */
int fsagg_upload_h2d(void *dst, const void *src, size_t nbytes, void *stage,
                     int slot, int nslot, fsagg_stream_t copy_stream,
                     fsagg_stream_t consumer);
int fsagg_upload_wait(int slot, fsagg_stream_t stream);
/* A kernel copies `n` 8-byte words from pinned, device-mapped host memory
 * `host_src` (hipHostMalloc / torch pin_memory) into device `dst` on
 * `stream` — capturable into a HIP graph, so a replayed launch chain reads
 * its per-call row table from a fixed pinned buffer that the host refills
 * before each replay (no copy-engine call per replay). */
int fsagg_fetch_mapped_u64(const void *host_src, void *dst, int64_t n,
                           fsagg_stream_t stream);
int fsagg_weighted_sum_hosttab_f32(const uint64_t *rows,
                                   const float *weights,
                                   const float *prescale, int n,
                                   int64_t numel, const float *base,
                                   float *const *outs, int nout,
                                   fsagg_stream_t stream);
/* fsagg_weighted_sum_rows_f32 with the row set's tables on the HOST, in
 * the launch's kernel arguments: `tab` the segment-major [nseg][n] virtual
 * bases (fsagg_rows' tab with ss = n; 0 = a client lacking the key),
 * `weights` / `prescale` (NULL: none) n floats, `base` (NULL: none) nseg
 * virtual bases of the init model; n <= FSAGG_HOSTTAB_ROWS_MAX_CLIENTS,
 * n·nseg <= FSAGG_HOSTTAB_ROWS_MAX_PTRS, nseg <= FSAGG_HOSTTAB_ROWS_MAX_SEGS
 * with a base.  `chunks` / `chunk_elems` as for fsagg_weighted_sum_rows_f32
 * (a device chunk list, cached per layout).  Same arithmetic, bit for bit.
 * For small multi-key row sets whose per-call table uploads cost more host
 * time than the kernel: a multi-Krum selection's average over fresh
 * uploads (krum_aggregator.py:81-90 through the weighted sum). */
#define FSAGG_HOSTTAB_ROWS_MAX_CLIENTS 64
#define FSAGG_HOSTTAB_ROWS_MAX_PTRS 256
#define FSAGG_HOSTTAB_ROWS_MAX_SEGS 64
int fsagg_weighted_sum_rows_hosttab_f32(const uint64_t *tab, int n, int nseg,
                                        const fsagg_chunk *chunks, int nchunk,
                                        int64_t chunk_elems,
                                        const float *weights,
                                        const float *prescale,
                                        const uint64_t *base, float *out,
                                        fsagg_stream_t stream);
/* Krum's certified selection on the device (krum_aggregator.py:75-90):
 * from the Gram chain's finish buffer `buf` (int32 [5][n][n]: D64, D, the
 * flags, B — fsagg_pairgram_rows_f32's outputs laid out as the Python
 * layer's ops._gram_buf), the scores over D64 (the sum of each row's
 * n − f − 2 smallest), their stable order and the certificate of the
 * first m (`ordered`: their order too) against the per-pair bounds —
 * csrc/host/krumcert.cpp's, on the device.  Writes `sel` (int32 [2 + n]:
 * certified, valid — no flagged pair and n − f − 2 > 0 —, then the order)
 * and, for the first min(m, n) clients in that order, the row-set table
 * `sub_tab` ([nsegt][msel] from `tab`, the clients' device table [nsegt][n]
 * with ss = n, or [1][n] with ss = 0), fp32 weights `sub_w` (fedavg
 * weights of their `sizes`, host fp64 [n]; 1/msel with ignore_weight) and,
 * with a `base` (host array of nseg device virtual bases), `sub_base`
 * (int64 [nseg]) — the operands of fsagg_weighted_sum_rows_f32, which the
 * caller launches behind this call without waiting for the host.
 * `work`: device fp64 [4n].  n <= FSAGG_KRUMSEL_MAX_CLIENTS, nseg <=
 * FSAGG_KRUMSEL_MAX_SEGS with a base. */
#define FSAGG_KRUMSEL_MAX_CLIENTS 256
#define FSAGG_KRUMSEL_MAX_SEGS 64
int fsagg_krum_select_f32(const int32_t *buf, int n, int nseg, int f, int m,
                          int ordered, const double *sizes, int ignore_weight,
                          const float *const *base, const int64_t *tab,
                          int64_t ss, int nsegt, double *work, int32_t *sel,
                          int64_t *sub_tab, float *sub_w, int64_t *sub_base,
                          fsagg_stream_t stream);
size_t fsagg_peer_handle_bytes(void);
int fsagg_peer_alloc(int device, size_t bytes, void **ptr);
int fsagg_peer_free(int device, void *ptr);
int fsagg_peer_status_alloc(void **host, void **dev);
int fsagg_peer_status_free(void *host);
int fsagg_peer_handle(void *ptr, void *handle);
int fsagg_peer_open(int device, const void *handle, void **ptr);
int fsagg_peer_close(int device, void *ptr);
int fsagg_peer_pci_bus_id(int device, char *buf, int len);
int fsagg_peer_can_access(int device, const char *peer_bus_id);
int fsagg_weighted_sum_bcast_f32(const float *const *rows,
                                 const float *weights, const float *prescale,
                                 int n, int64_t numel, const float *base,
                                 float *const *outs, int nout,
                                 fsagg_stream_t stream);
int fsagg_peer_push_f32(const float *src, float *const *dsts, int ndst,
                        int64_t n, fsagg_stream_t stream);
int fsagg_peer_barrier(uint32_t *const *flags, int world, int rank,
                       uint32_t epoch, uint64_t timeout_ticks,
                       uint32_t *status, fsagg_stream_t stream);

/*
 * Deterministic synthetic client updates (benchmarks / tests): fills the
 * [n][ld] slab X with u = hash(seed, client, index) mapped to [-1, 1),
 * index < numel; the same generator is restated on the host by the tests.
 */
int fsagg_fill_uniform_f32(float *X, int n, int64_t numel, int64_t ld,
                           uint64_t seed, int64_t index_offset,
                           fsagg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FSAGG_H_ */

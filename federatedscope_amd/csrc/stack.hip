// Staging of device-resident client updates into the client stack (gfx950).
//
// The reference's aggregators take one state_dict per client; when those
// tensors already live in HBM (GPU trainers, the loopback simulator), the
// per-key copies into the stack's rows were the whole cost of a robust
// aggregate() call (200 clients × 12 keys = 2400 copy launches ≈ 20 ms
// against a 1.5 ms median).  One launch does them all: the host lists the
// bucket as chunks of at most kChunk coordinates that never straddle a key
// (built once per layout), and block (chunk c, client i) copies
// src[i][key(c)][start(c) ...] into row i at the key's offset.  A NULL source
// (a key the client does not carry) leaves the row untouched.  HBM-bound: 4 B
// read + 4 B written per coordinate.
#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;
constexpr int kChunk = FSAGG_STACK_CHUNK;
constexpr int kPer = kChunk / kBlock;  // coordinates per lane (8)

__global__ __launch_bounds__(kBlock) void gather_rows_kernel(
    const float *const *__restrict__ src, int nseg,
    float *const *__restrict__ dst_rows, const int64_t *__restrict__ key_off,
    const int64_t *__restrict__ key_len, const int32_t *__restrict__ chunk_key,
    const int64_t *__restrict__ chunk_start) {
  const int c = blockIdx.x, i = blockIdx.y;
  const int s = chunk_key[c];
  const float *x = src[int64_t(i) * nseg + s];
  if (!x) return;  // key absent from this client
  const int64_t start = chunk_start[c];
  const int64_t rem = key_len[s] - start;
  const int len = rem < kChunk ? int(rem) : kChunk;
  x += start;
  float *y = dst_rows[i] + key_off[s] + start;
  float v[kPer];
  if (len == kChunk) {  // all loads in flight, then the stores
#pragma unroll
    for (int e = 0; e < kPer; ++e) v[e] = gload_nt(x + e * kBlock + threadIdx.x);
#pragma unroll
    for (int e = 0; e < kPer; ++e) y[e * kBlock + threadIdx.x] = v[e];
  } else {
    for (int q = threadIdx.x; q < len; q += kBlock) y[q] = gld(x + q);
  }
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_gather_rows_f32(const float *const *src, int n, int nseg,
                                     float *const *dst_rows,
                                     const int64_t *key_off,
                                     const int64_t *key_len,
                                     const int32_t *chunk_key,
                                     const int64_t *chunk_start, int nchunk,
                                     fsagg_stream_t stream) {
  if (!src || !dst_rows || !key_off || !key_len || !chunk_key ||
      !chunk_start || n < 0 || nseg < 1 || nchunk < 0 || n > 65535) {
    set_error("fsagg_gather_rows_f32: invalid argument (n=%d nseg=%d "
              "nchunk=%d)", n, nseg, nchunk);
    return FSAGG_EINVAL;
  }
  if (n == 0 || nchunk == 0) return FSAGG_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(unsigned(nchunk), unsigned(n)),
                     dim3(kBlock), 0, as_stream(stream), src, nseg, dst_rows,
                     key_off, key_len, chunk_key, chunk_start);
  return check_launch("fsagg_gather_rows_f32");
}

// ---------------------------------------------------------------------------
// fsagg_fetch_mapped_u64: a kernel copies n 8-byte words from pinned
// (device-mapped) host memory into device memory.  Captured as the first
// node of a launch chain's HIP graph it replaces a per-call hipMemcpyAsync
// of the chain's row table (~19 µs of host time through the upload ring):
// the host writes the table into the fixed pinned buffer and replays, and
// the graph's own kernel reads it over PCIe (coherent host memory, a few
// KiB, one 8-B load per lane).
// ---------------------------------------------------------------------------
namespace fsagg {
namespace {
__global__ __launch_bounds__(kBlock) void fetch_mapped_kernel(
    const uint64_t *__restrict__ src, uint64_t *__restrict__ dst, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * kBlock)
    dst[i] = __builtin_nontemporal_load(src + i);
}
}  // namespace
}  // namespace fsagg

extern "C" int fsagg_fetch_mapped_u64(const void *host_src, void *dst,
                                      int64_t n, fsagg_stream_t stream) {
  if (!host_src || !dst || n < 0) {
    set_error("fsagg_fetch_mapped_u64: invalid argument (n=%lld)",
              (long long)n);
    return FSAGG_EINVAL;
  }
  if (n == 0) return FSAGG_OK;
  void *dsrc = nullptr;
  const hipError_t e =
      hipHostGetDevicePointer(&dsrc, const_cast<void *>(host_src), 0);
  if (e != hipSuccess || !dsrc) {
    set_error("fsagg_fetch_mapped_u64: not device-mapped host memory (%s)",
              hipGetErrorString(e));
    return FSAGG_EINVAL;
  }
  int64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 64) blocks = 64;
  hipLaunchKernelGGL(fetch_mapped_kernel, dim3(unsigned(blocks)),
                     dim3(kBlock), 0, as_stream(stream),
                     static_cast<const uint64_t *>(dsrc),
                     static_cast<uint64_t *>(dst), n);
  return check_launch("fsagg_fetch_mapped_u64");
}

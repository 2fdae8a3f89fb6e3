// Peer assembly over xGMI (gfx950): the strong-scaled aggregation writes
// its result straight into every GPU's copy of the output
// (fsagg_weighted_sum_bcast_f32), then one tiny flag barrier tells each GPU
// that every peer's stores have landed.  SURVEY §8(e): the cross-GPU step is
// a concatenation of disjoint parameter ranges, never an arithmetic reduce.
//
// Memory: the output copies and the flag arrays are allocated uncached
// (hipDeviceMallocUncached), so every GPU's stores and loads of them go to
// the owning GPU's memory instead of a local L2 that a peer's xGMI stores
// would not invalidate.  Buffers are exported with hipIpcGetMemHandle and
// imported by the peer processes (one process per GPU).
//
// Replaces the reference's device-resident multi-GPU traffic: per-key
// dist.send/recv of model tensors between the server rank and client ranks
// (federatedscope/core/communication.py:61-76,
// core/parallel/parallel_runner.py:22-24,243-302).
#include "common.h"

namespace fsagg {
namespace {

struct Flags {
  uint32_t *p[FSAGG_MAX_PEERS];  // p[r] = rank r's flag array (world words)
};

// One workgroup.  Lane t < world stores `epoch` into rank t's flag word for
// this rank, then waits until this rank's word for rank t reaches `epoch`.
// The flag words are uncached; the stores are release and the loads acquire
// at system scope.  The spin is bounded: after `timeout` ticks of the
// 100 MHz constant clock the lane sets status[0] and gives up, so the grid
// always drains (a lost peer becomes an error the host reads, not a hang).
// Last, lane 0 stores `epoch` into status[1]: the host (status in mapped
// pinned memory) sees the barrier done without an event or a copy.
__global__ void peer_barrier_kernel(Flags f, int world, int rank,
                                    uint32_t epoch, uint64_t timeout,
                                    uint32_t *status) {
  const int t = threadIdx.x;
  if (t < world) {
    __hip_atomic_store(f.p[t] + rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t *mine = f.p[rank] + t;
    const uint64_t t0 = wall_clock64();
    while (int32_t(__hip_atomic_load(mine, __ATOMIC_ACQUIRE,
                                     __HIP_MEMORY_SCOPE_SYSTEM) -
                   epoch) < 0) {
      if (wall_clock64() - t0 > timeout) {
        __hip_atomic_store(status, 1u + uint32_t(t), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  if (t == 0)
    __hip_atomic_store(status + 1, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Dsts {
  float *p[FSAGG_MAX_PEERS];
};

// The peer assembly's epilogue for reductions without a fused broadcast
// (order statistics, row-set averages): this rank's finished piece is read
// once and stored into each peer's copy (16-B vector stores over xGMI).
__global__ __launch_bounds__(256) void peer_push_kernel(const float *src,
                                                        Dsts d, int nd,
                                                        int64_t n) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const int64_t n4 = n / 4;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4 *>(src)[i];
    for (int k = 0; k < nd; ++k) reinterpret_cast<f32x4 *>(d.p[k])[i] = v;
  }
  const int64_t t = 4 * n4 + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t < n)
    for (int k = 0; k < nd; ++k) d.p[k][t] = src[t];
}

int hip_fail(const char *what, hipError_t e) {
  set_error("%s: %s", what, hipGetErrorString(e));
  return FSAGG_EHIP;
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" size_t fsagg_peer_handle_bytes(void) {
  return sizeof(hipIpcMemHandle_t);
}

extern "C" int fsagg_peer_alloc(int device, size_t bytes, void **ptr) {
  if (!ptr || bytes == 0) {
    set_error("fsagg_peer_alloc: invalid argument");
    return FSAGG_EINVAL;
  }
  *ptr = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail("fsagg_peer_alloc: hipSetDevice", e);
  e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess)
    return hip_fail("fsagg_peer_alloc: hipExtMallocWithFlags", e);
  e = hipMemset(*ptr, 0, bytes);
  if (e != hipSuccess) return hip_fail("fsagg_peer_alloc: hipMemset", e);
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail("fsagg_peer_alloc: sync", e);
  return FSAGG_OK;
}

extern "C" int fsagg_peer_free(int device, void *ptr) {
  if (!ptr) return FSAGG_OK;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail("fsagg_peer_free: hipSetDevice", e);
  e = hipFree(ptr);
  if (e != hipSuccess) return hip_fail("fsagg_peer_free: hipFree", e);
  return FSAGG_OK;
}

extern "C" int fsagg_peer_status_alloc(void **host, void **dev) {
  if (!host || !dev) {
    set_error("fsagg_peer_status_alloc: invalid argument");
    return FSAGG_EINVAL;
  }
  *host = *dev = nullptr;
  hipError_t e = hipHostMalloc(host, 64, hipHostMallocMapped);
  if (e != hipSuccess)
    return hip_fail("fsagg_peer_status_alloc: hipHostMalloc", e);
  std::memset(*host, 0, 64);
  e = hipHostGetDevicePointer(dev, *host, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(*host);
    *host = nullptr;
    return hip_fail("fsagg_peer_status_alloc: hipHostGetDevicePointer", e);
  }
  return FSAGG_OK;
}

extern "C" int fsagg_peer_status_free(void *host) {
  if (!host) return FSAGG_OK;
  hipError_t e = hipHostFree(host);
  if (e != hipSuccess) return hip_fail("fsagg_peer_status_free", e);
  return FSAGG_OK;
}

extern "C" int fsagg_peer_handle(void *ptr, void *handle) {
  if (!ptr || !handle) {
    set_error("fsagg_peer_handle: invalid argument");
    return FSAGG_EINVAL;
  }
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e != hipSuccess) return hip_fail("fsagg_peer_handle", e);
  std::memcpy(handle, &h, sizeof(h));
  return FSAGG_OK;
}

extern "C" int fsagg_peer_open(int device, const void *handle, void **ptr) {
  if (!handle || !ptr) {
    set_error("fsagg_peer_open: invalid argument");
    return FSAGG_EINVAL;
  }
  *ptr = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail("fsagg_peer_open: hipSetDevice", e);
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  e = hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) return hip_fail("fsagg_peer_open", e);
  return FSAGG_OK;
}

extern "C" int fsagg_peer_close(int device, void *ptr) {
  if (!ptr) return FSAGG_OK;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail("fsagg_peer_close: hipSetDevice", e);
  e = hipIpcCloseMemHandle(ptr);
  if (e != hipSuccess) return hip_fail("fsagg_peer_close", e);
  return FSAGG_OK;
}

extern "C" int fsagg_peer_pci_bus_id(int device, char *buf, int len) {
  if (!buf || len < 16) {
    set_error("fsagg_peer_pci_bus_id: invalid argument");
    return FSAGG_EINVAL;
  }
  hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
  if (e != hipSuccess) return hip_fail("fsagg_peer_pci_bus_id", e);
  return FSAGG_OK;
}

extern "C" int fsagg_peer_can_access(int device, const char *peer_bus_id) {
  if (!peer_bus_id) {
    set_error("fsagg_peer_can_access: invalid argument");
    return FSAGG_EINVAL;
  }
  int peer = -1;
  if (hipDeviceGetByPCIBusId(&peer, peer_bus_id) != hipSuccess || peer < 0) {
    (void)hipGetLastError();
    return 2;  // the peer's GPU is not visible here: nothing to check
  }
  if (peer == device) return 1;
  int ok = 0;
  hipError_t e = hipDeviceCanAccessPeer(&ok, device, peer);
  if (e != hipSuccess) return hip_fail("fsagg_peer_can_access", e);
  return ok ? 1 : 0;
}

extern "C" int fsagg_peer_push_f32(const float *src, float *const *dsts,
                                   int ndst, int64_t n,
                                   fsagg_stream_t stream) {
  if (!src || !dsts || ndst < 0 || ndst > FSAGG_MAX_PEERS || n < 0 ||
      !aligned16(src)) {
    set_error("fsagg_peer_push_f32: invalid argument (ndst=%d n=%lld)", ndst,
              static_cast<long long>(n));
    return FSAGG_EINVAL;
  }
  Dsts d{};
  for (int k = 0; k < ndst; ++k) {
    if (!dsts[k] || !aligned16(dsts[k])) {
      set_error("fsagg_peer_push_f32: destination %d is NULL or not 16-byte "
                "aligned", k);
      return FSAGG_EINVAL;
    }
    d.p[k] = dsts[k];
  }
  if (n == 0 || ndst == 0) return FSAGG_OK;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4 * int64_t(device_cu_count())) blocks = 4 * device_cu_count();
  hipLaunchKernelGGL(peer_push_kernel, dim3(unsigned(blocks)), dim3(256), 0,
                     as_stream(stream), src, d, ndst, n);
  return check_launch("fsagg_peer_push_f32");
}

extern "C" int fsagg_peer_barrier(uint32_t *const *flags, int world, int rank,
                                  uint32_t epoch, uint64_t timeout_ticks,
                                  uint32_t *status, fsagg_stream_t stream) {
  if (!flags || !status || world < 1 || world > FSAGG_MAX_PEERS || rank < 0 ||
      rank >= world) {
    set_error("fsagg_peer_barrier: invalid argument (world=%d rank=%d)",
              world, rank);
    return FSAGG_EINVAL;
  }
  Flags f{};
  for (int r = 0; r < world; ++r) {
    if (!flags[r]) {
      set_error("fsagg_peer_barrier: flag array %d is NULL", r);
      return FSAGG_EINVAL;
    }
    f.p[r] = flags[r];
  }
  hipLaunchKernelGGL(peer_barrier_kernel, dim3(1), dim3(kWave), 0,
                     as_stream(stream), f, world, rank, epoch, timeout_ticks,
                     status);
  return check_launch("fsagg_peer_barrier");
}

// Error plumbing shared by every libfsagg entry point.
#include <cstdarg>
#include <mutex>

#include "common.h"

namespace fsagg {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return FSAGG_EHIP;
  }
  return FSAGG_OK;
}

int device_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                              dev) != hipSuccess || cus <= 0)
      cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

}  // namespace fsagg

// ---------------------------------------------------------------------------
// Small-table uploads (fsagg_upload_h2d): the caller's pinned staging ring
// and device ring share a slot index; the library keeps two events per slot
// and device — `done` (the copy out of the slot has run: the pinned slot
// may be refilled) and `mark` (recorded on the consumer stream at upload j:
// everything enqueued on it before that upload).  Reusing device slot s at
// upload j, the copy stream first waits for the mark of upload j − nslot/2,
// i.e. for every consumer enqueued within nslot/2 uploads of slot s's
// previous upload, so a table is never overwritten under a kernel still
// reading it.
// ---------------------------------------------------------------------------
namespace fsagg {
namespace {
constexpr int kUpMaxSlots = 256;
constexpr int kUpMaxDevs = 64;
struct UpEvents {
  hipEvent_t done[kUpMaxSlots];
  hipEvent_t mark[kUpMaxSlots];
  bool used_done[kUpMaxSlots];
  bool used_mark[kUpMaxSlots];
  bool ready;
};
UpEvents g_up[kUpMaxDevs];
std::mutex g_up_mu;
}  // namespace
}  // namespace fsagg

extern "C" int fsagg_upload_h2d(void *dst, const void *src, size_t nbytes,
                                void *stage, int slot, int nslot,
                                fsagg_stream_t copy_stream,
                                fsagg_stream_t consumer) {
  using namespace fsagg;
  if (!dst || (!src && nbytes) || !stage || nslot < 2 ||
      nslot > kUpMaxSlots || slot < 0 || slot >= nslot) {
    set_error("fsagg_upload_h2d: invalid argument (slot %d of %d)", slot,
              nslot);
    return FSAGG_EINVAL;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kUpMaxDevs) {
    set_error("fsagg_upload_h2d: no current device");
    return FSAGG_EHIP;
  }
  std::lock_guard<std::mutex> lock(g_up_mu);
  UpEvents &E = g_up[dev];
  if (!E.ready) {
    for (int i = 0; i < kUpMaxSlots; ++i) {
      if (hipEventCreateWithFlags(&E.done[i], hipEventDisableTiming) !=
              hipSuccess ||
          hipEventCreateWithFlags(&E.mark[i], hipEventDisableTiming) !=
              hipSuccess) {
        set_error("fsagg_upload_h2d: hipEventCreate failed");
        return FSAGG_EHIP;
      }
      E.used_done[i] = E.used_mark[i] = false;
    }
    E.ready = true;
  }
  hipStream_t cs = as_stream(copy_stream), us = as_stream(consumer);
  // the pinned slot's previous copy has run
  if (E.used_done[slot] && hipEventSynchronize(E.done[slot]) != hipSuccess) {
    set_error("fsagg_upload_h2d: hipEventSynchronize failed");
    return FSAGG_EHIP;
  }
  if (nbytes) std::memcpy(stage, src, nbytes);
  const int lag = (slot + nslot / 2) % nslot;
  hipError_t e = hipSuccess;
  if (E.used_mark[lag]) e = hipStreamWaitEvent(cs, E.mark[lag], 0);
  if (e == hipSuccess && nbytes)
    e = hipMemcpyAsync(dst, stage, nbytes, hipMemcpyHostToDevice, cs);
  if (e == hipSuccess) e = hipEventRecord(E.done[slot], cs);
  if (e == hipSuccess) e = hipStreamWaitEvent(us, E.done[slot], 0);
  if (e == hipSuccess) e = hipEventRecord(E.mark[slot], us);
  if (e != hipSuccess) {
    set_error("fsagg_upload_h2d: %s", hipGetErrorString(e));
    return FSAGG_EHIP;
  }
  E.used_done[slot] = E.used_mark[slot] = true;
  return FSAGG_OK;
}

// a stream that was not the upload's consumer waits for slot `slot`'s copy
// (the done event of the slot's latest copy, on the same copy stream, so it
// completes after this one)
extern "C" int fsagg_upload_wait(int slot, fsagg_stream_t stream) {
  using namespace fsagg;
  int dev = 0;
  if (slot < 0 || slot >= kUpMaxSlots || hipGetDevice(&dev) != hipSuccess ||
      dev < 0 || dev >= kUpMaxDevs) {
    set_error("fsagg_upload_wait: invalid argument");
    return FSAGG_EINVAL;
  }
  std::lock_guard<std::mutex> lock(g_up_mu);
  UpEvents &E = g_up[dev];
  if (!E.ready || !E.used_done[slot]) return FSAGG_OK;
  if (hipStreamWaitEvent(as_stream(stream), E.done[slot], 0) != hipSuccess) {
    set_error("fsagg_upload_wait: hipStreamWaitEvent failed");
    return FSAGG_EHIP;
  }
  return FSAGG_OK;
}

extern "C" int fsagg_version(void) { return FSAGG_VERSION; }

extern "C" const char *fsagg_last_error(void) { return fsagg::g_err; }

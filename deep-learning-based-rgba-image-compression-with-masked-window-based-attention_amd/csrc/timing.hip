// Kernel timing helpers for bench.py's launch profiler (not on the compute path).
//
// HIP events created with hipEventDisableSystemFence: recording them performs no
// system-scope cache writeback/invalidate, so bracketing every launch does not cold-start
// the L2 of the next kernel (torch.cuda.Event's default events do, inflating per-kernel
// times).  (Recording on a capturing stream asks for an external event node,
// hipEventRecordExternal; ROCm 7.0 rejects that, so bench.py times eager launches.)
#include "common.h"

extern "C" int rgbac_timer_create(void** ev) {
  RGBAC_REQUIRE(ev != nullptr, "null event slot");
  hipEvent_t e;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
    rgbac::set_error("hipEventCreateWithFlags failed");
    return RGBAC_E_LAUNCH;
  }
  *ev = reinterpret_cast<void*>(e);
  return RGBAC_OK;
}

extern "C" int rgbac_timer_record(void* ev, void* stream) {
  RGBAC_REQUIRE(ev != nullptr, "null event");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
  const unsigned flags = cs == hipStreamCaptureStatusActive ? hipEventRecordExternal : 0u;
  if (hipEventRecordWithFlags(reinterpret_cast<hipEvent_t>(ev), st, flags) != hipSuccess) {
    rgbac::set_error("hipEventRecordWithFlags failed");
    return RGBAC_E_LAUNCH;
  }
  return RGBAC_OK;
}

extern "C" int rgbac_timer_elapsed_ms(void* start, void* stop, float* ms) {
  RGBAC_REQUIRE(start && stop && ms, "null argument");
  if (hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start),
                          reinterpret_cast<hipEvent_t>(stop)) != hipSuccess) {
    rgbac::set_error("hipEventElapsedTime failed");
    return RGBAC_E_LAUNCH;
  }
  return RGBAC_OK;
}

extern "C" int rgbac_timer_destroy(void* ev) {
  if (ev) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev));
  return RGBAC_OK;
}

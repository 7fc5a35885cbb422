// Gradient exchange of the data-parallel training step (the reference trains
// on one GPU -- DataParallel is commented out at trainRGB.py:374 -- so this has no reference
// counterpart: it is the all-reduce the build adds for BASELINE config 5).
//
// RCCL is called directly, not through torch.distributed's ProcessGroup: a bucket all-reduce
// is ONE ncclAllReduce on the caller's stream, with no Python work object, no watchdog thread
// polling events, and nothing that breaks when the training step -- backward, the bucket
// all-reduces it launches, clamp + Adam -- is captured in a HIP graph and replayed (RCCL
// collectives are stream-ordered and capturable).  torch.distributed stays the bootstrap:
// it carries the 128-byte unique id from rank 0 to the other ranks.
//
// The library is the one PyTorch itself loaded (its bundled librccl.so, path from the host
// side): it is dlopen'ed here and called through function pointers, so this process holds
// exactly one RCCL (no second copy of the NCCL symbols next to torch's).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "common.h"

namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
};

Rccl g_rccl;

int nccl_fail(const char* what, ncclResult_t r) {
  std::string msg = std::string(what) + ": RCCL error " + std::to_string((int)r);
  if (g_rccl.error_string) msg += std::string(" (") + g_rccl.error_string(r) + ")";
  rgbac::set_error(msg);
  return RGBAC_E_LAUNCH;
}

}  // namespace

extern "C" int rgbac_comm_load(const char* librccl_path) {
  RGBAC_REQUIRE(librccl_path != nullptr, "null library path");
  if (g_rccl.handle) return RGBAC_OK;
  void* h = dlopen(librccl_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    rgbac::set_error(std::string("rgbac_comm_load: dlopen failed: ") + dlerror());
    return RGBAC_E_ARG;
  }
  Rccl r;
  r.handle = h;
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
  r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
  r.comm_count = reinterpret_cast<decltype(r.comm_count)>(dlsym(h, "ncclCommCount"));
  r.async_error = reinterpret_cast<decltype(r.async_error)>(dlsym(h, "ncclCommGetAsyncError"));
  r.comm_abort = reinterpret_cast<decltype(r.comm_abort)>(dlsym(h, "ncclCommAbort"));
  if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy ||
      !r.error_string || !r.comm_count || !r.async_error || !r.comm_abort) {
    dlclose(h);
    rgbac::set_error("rgbac_comm_load: the library lacks an NCCL entry point");
    return RGBAC_E_ARG;
  }
  g_rccl = r;
  return RGBAC_OK;
}

extern "C" int rgbac_comm_unique_id(void* id_out) {
  RGBAC_REQUIRE(g_rccl.handle, "rgbac_comm_load first");
  RGBAC_REQUIRE(id_out != nullptr, "null id buffer");
  ncclUniqueId id;
  const ncclResult_t r = g_rccl.get_unique_id(&id);
  if (r != ncclSuccess) return nccl_fail("ncclGetUniqueId", r);
  memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return RGBAC_OK;
}

extern "C" int rgbac_comm_init(const void* id_in, int world, int rank, int device, void** comm) {
  RGBAC_REQUIRE(g_rccl.handle, "rgbac_comm_load first");
  RGBAC_REQUIRE(id_in && comm, "null pointer");
  RGBAC_REQUIRE(world >= 1 && rank >= 0 && rank < world, "rank / world");
  if (hipSetDevice(device) != hipSuccess) {
    rgbac::set_error("rgbac_comm_init: hipSetDevice failed");
    return RGBAC_E_ARG;
  }
  ncclUniqueId id;
  memcpy(id.internal, id_in, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = g_rccl.comm_init_rank(&c, world, id, rank);
  if (r != ncclSuccess) return nccl_fail("ncclCommInitRank", r);
  *comm = c;
  return RGBAC_OK;
}

extern "C" int rgbac_comm_allreduce_sum(void* comm, int dtype, void* buf, int64_t count,
                                        void* stream) {
  RGBAC_REQUIRE(g_rccl.handle && comm, "no communicator");
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(buf != nullptr && count >= 0, "buffer");
  if (count == 0) return RGBAC_OK;
  const ncclResult_t r =
      g_rccl.all_reduce(buf, buf, (size_t)count, dtype == RGBAC_F32 ? ncclFloat32 : ncclBfloat16,
                        ncclSum, reinterpret_cast<ncclComm_t>(comm),
                        reinterpret_cast<hipStream_t>(stream));
  if (r != ncclSuccess) return nccl_fail("ncclAllReduce", r);
  return RGBAC_OK;
}

extern "C" int rgbac_comm_destroy(void* comm) {
  RGBAC_REQUIRE(g_rccl.handle, "rgbac_comm_load first");
  if (!comm) return RGBAC_OK;
  const ncclResult_t r = g_rccl.comm_destroy(reinterpret_cast<ncclComm_t>(comm));
  if (r != ncclSuccess) return nccl_fail("ncclCommDestroy", r);
  return RGBAC_OK;
}

// Ranks the communicator itself spans (ncclCommCount): what a multi-GPU bench line reports as
// the world RCCL saw, independent of torch.distributed's view.
extern "C" int rgbac_comm_count(void* comm, int* count) {
  RGBAC_REQUIRE(g_rccl.handle && comm, "no communicator");
  RGBAC_REQUIRE(count != nullptr, "null count");
  const ncclResult_t r = g_rccl.comm_count(reinterpret_cast<ncclComm_t>(comm), count);
  if (r != ncclSuccess) return nccl_fail("ncclCommCount", r);
  return RGBAC_OK;
}

// Asynchronous error state of the communicator (ncclCommGetAsyncError): *err = 0 while healthy,
// else the ncclResult_t code (a peer died, a network / xGMI failure).  Polled from a host thread
// between steps (rgbac.parallel.CommWatchdog); a collective that can never complete otherwise
// blocks its stream -- and every rank's graph replay -- forever.
extern "C" int rgbac_comm_async_error(void* comm, int* err) {
  RGBAC_REQUIRE(g_rccl.handle && comm, "no communicator");
  RGBAC_REQUIRE(err != nullptr, "null error out");
  ncclResult_t a = ncclSuccess;
  const ncclResult_t r = g_rccl.async_error(reinterpret_cast<ncclComm_t>(comm), &a);
  if (r != ncclSuccess) return nccl_fail("ncclCommGetAsyncError", r);
  *err = (int)a;
  return RGBAC_OK;
}

// Abort the communicator (ncclCommAbort): kernels of pending collectives are released and the
// handle is freed.  The host then exits the process non-zero; nothing here restarts anything.
extern "C" int rgbac_comm_abort(void* comm) {
  RGBAC_REQUIRE(g_rccl.handle, "rgbac_comm_load first");
  if (!comm) return RGBAC_OK;
  const ncclResult_t r = g_rccl.comm_abort(reinterpret_cast<ncclComm_t>(comm));
  if (r != ncclSuccess) return nccl_fail("ncclCommAbort", r);
  return RGBAC_OK;
}

// RCCL entry points of the C-ABI (include/pwg.h): the design's ONE collective, a broadcast of the
// packed weight image from a root rank to every rank over xGMI, plus the
// communicator helpers a host without torch.distributed needs to set it up.
//
// librccl is resolved at first use with dlopen (soname librccl.so.1), so the library loads and runs
// single-GPU work on machines without RCCL, and inside a torch process it binds to the RCCL torch
// already mapped (same soname: one RCCL per process). Only rccl.h's TYPES are used at compile time.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string>

#include "../../include/pwg.h"
#include "pwg_internal.h"

namespace {

struct Rccl {
  bool tried = false;
  void* so = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl g_rccl;
std::mutex g_rccl_mu;

int rccl(Rccl** out) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!g_rccl.tried) {
    g_rccl.tried = true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
      if ((g_rccl.so = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
    if (g_rccl.so) {
      g_rccl.get_unique_id = reinterpret_cast<decltype(g_rccl.get_unique_id)>(dlsym(g_rccl.so, "ncclGetUniqueId"));
      g_rccl.comm_init_rank = reinterpret_cast<decltype(g_rccl.comm_init_rank)>(dlsym(g_rccl.so, "ncclCommInitRank"));
      g_rccl.comm_destroy = reinterpret_cast<decltype(g_rccl.comm_destroy)>(dlsym(g_rccl.so, "ncclCommDestroy"));
      g_rccl.broadcast = reinterpret_cast<decltype(g_rccl.broadcast)>(dlsym(g_rccl.so, "ncclBroadcast"));
      g_rccl.error_string = reinterpret_cast<decltype(g_rccl.error_string)>(dlsym(g_rccl.so, "ncclGetErrorString"));
    }
  }
  if (!g_rccl.get_unique_id || !g_rccl.comm_init_rank || !g_rccl.comm_destroy || !g_rccl.broadcast)
    return pwg::set_error(PWG_ERR_UNSUPPORTED, "RCCL (librccl.so.1) is not available in this process");
  *out = &g_rccl;
  return PWG_OK;
}

int rccl_fail(Rccl* r, ncclResult_t e, const char* what) {
  std::string m = std::string(what) + ": RCCL error " + std::to_string((int)e);
  if (r->error_string) m += std::string(" (") + r->error_string(e) + ")";
  return pwg::set_error(PWG_ERR_HIP, m.c_str());
}

}  // namespace

extern "C" {

int pwg_rccl_unique_id(void* id_out) {
  if (!id_out) return pwg::set_error(PWG_ERR_INVALID, "null argument");
  Rccl* r = nullptr;
  if (int rc = rccl(&r)) return rc;
  ncclUniqueId id;
  const ncclResult_t e = r->get_unique_id(&id);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
  static_assert(sizeof(ncclUniqueId) == PWG_RCCL_UNIQUE_ID_BYTES, "ncclUniqueId size");
  __builtin_memcpy(id_out, &id, sizeof(id));
  return PWG_OK;
}

int pwg_rccl_comm_create(int nranks, const void* id, int rank, int device, void** comm_out) {
  if (!id || !comm_out) return pwg::set_error(PWG_ERR_INVALID, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return pwg::set_error(PWG_ERR_INVALID, "rank out of range");
  Rccl* r = nullptr;
  if (int rc = rccl(&r)) return rc;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
    return pwg::set_error(PWG_ERR_HIP, "hipSetDevice failed");
  ncclUniqueId uid;
  __builtin_memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm = nullptr;
  const ncclResult_t e = r->comm_init_rank(&comm, nranks, uid, rank);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommInitRank");
  *comm_out = comm;
  return PWG_OK;
}

int pwg_rccl_comm_destroy(void* comm) {
  if (!comm) return PWG_OK;
  Rccl* r = nullptr;
  if (int rc = rccl(&r)) return rc;
  const ncclResult_t e = r->comm_destroy(static_cast<ncclComm_t>(comm));
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclCommDestroy");
  return PWG_OK;
}

int pwg_broadcast_weights(const PwgHandle* h, void* comm, int root, float* packed, void* stream) {
  if (!h || !comm || !packed) return pwg::set_error(PWG_ERR_INVALID, "null argument");
  Rccl* r = nullptr;
  if (int rc = rccl(&r)) return rc;
  const size_t n = (size_t)pwg_packed_weight_count(h);
  const ncclResult_t e =
      r->broadcast(packed, packed, n, ncclFloat32, root, static_cast<ncclComm_t>(comm), (hipStream_t)stream);
  if (e != ncclSuccess) return rccl_fail(r, e, "ncclBroadcast of the packed weights");
  return PWG_OK;
}

}  // extern "C"

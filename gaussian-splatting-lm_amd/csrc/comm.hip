// comm.hip -- RCCL collectives behind the C ABI ("gslm_allreduce* (RCCL comm handle passed in)").
//
// The multi-GPU LM product (gslm.parallel) moves its data with torch.distributed, whose "nccl" backend is RCCL; a
// host without torch drives the same exchanges through these entry points instead: a communicator made from a
// unique id that one rank creates and the host broadcasts (any channel), then in-place sum all-reduces of the CG
// scalars (f64) and of param-space partial products J^T r / J^T W J v (f32), the all-to-all of the
// Gaussian-sharded exchange and the all-gather of the screen exchange.  Every call is enqueued on the caller's stream and returns at once (RCCL's own
// stream semantics); the caller orders its kernels around it with the stream, as with any other launch.
//
// librccl is opened at the first communicator call (dlopen), not linked: the library loads and its compute entry
// points work on a host without RCCL, and in a torch process the dlopen returns the librccl that torch already
// mapped (one RCCL per process).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "gslm_internal.hpp"

namespace gslm {
namespace {

constexpr int kIdBytes = NCCL_UNIQUE_ID_BYTES;
static_assert(sizeof(ncclUniqueId) == kIdBytes, "RCCL unique id layout");

// the entry points used, resolved from the loaded librccl (types from rccl/rccl.h)
struct Rccl {
  void* so = nullptr;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclAllToAll) AllToAll = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "librccl.so"}) {
      r.so = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (r.so) break;
    }
    if (!r.so) return;
    r.GetUniqueId = reinterpret_cast<decltype(r.GetUniqueId)>(dlsym(r.so, "ncclGetUniqueId"));
    r.CommInitRank = reinterpret_cast<decltype(r.CommInitRank)>(dlsym(r.so, "ncclCommInitRank"));
    r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(dlsym(r.so, "ncclCommDestroy"));
    r.AllReduce = reinterpret_cast<decltype(r.AllReduce)>(dlsym(r.so, "ncclAllReduce"));
    r.AllToAll = reinterpret_cast<decltype(r.AllToAll)>(dlsym(r.so, "ncclAllToAll"));
    r.AllGather = reinterpret_cast<decltype(r.AllGather)>(dlsym(r.so, "ncclAllGather"));
    r.GetErrorString = reinterpret_cast<decltype(r.GetErrorString)>(dlsym(r.so, "ncclGetErrorString"));
  });
  if (!r.so || !r.GetUniqueId || !r.CommInitRank || !r.CommDestroy || !r.AllReduce || !r.AllToAll ||
      !r.AllGather) {
    set_error("RCCL unavailable: librccl.so.1 not found or missing an entry point");
    return nullptr;
  }
  return &r;
}

int rccl_status(const Rccl* r, ncclResult_t st, const char* who) {
  if (st == ncclSuccess) return GSLM_OK;
  set_error(std::string(who) + ": " + (r->GetErrorString ? r->GetErrorString(st) : "RCCL error"));
  return GSLM_ERR_HIP;
}

struct Comm {
  ncclComm_t c;
  int nranks, rank;
};

}  // namespace
}  // namespace gslm

using namespace gslm;

extern "C" {

int32_t gslm_comm_id_bytes(void) { return kIdBytes; }

int gslm_comm_unique_id(void* id_out) {
  if (!id_out) {
    set_error("comm_unique_id: NULL id_out");
    return GSLM_ERR_INVALID;
  }
  const Rccl* r = rccl();
  if (!r) return GSLM_ERR_HIP;
  ncclUniqueId id;
  const int st = rccl_status(r, r->GetUniqueId(&id), "ncclGetUniqueId");
  if (st) return st;
  std::memcpy(id_out, id.internal, kIdBytes);
  return GSLM_OK;
}

int gslm_comm_init(const void* id, int32_t nranks, int32_t rank, void** comm_out) {
  if (!id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("comm_init: NULL id / comm_out or rank outside [0, nranks)");
    return GSLM_ERR_INVALID;
  }
  *comm_out = nullptr;
  const Rccl* r = rccl();
  if (!r) return GSLM_ERR_HIP;
  ncclUniqueId rid;
  std::memcpy(rid.internal, id, kIdBytes);
  ncclComm_t c = nullptr;
  const int st = rccl_status(r, r->CommInitRank(&c, nranks, rid, rank), "ncclCommInitRank");
  if (st) return st;
  *comm_out = new Comm{c, nranks, rank};
  return GSLM_OK;
}

int gslm_comm_destroy(void* comm) {
  if (!comm) return GSLM_OK;
  Comm* cm = static_cast<Comm*>(comm);
  const Rccl* r = rccl();
  int st = GSLM_OK;
  if (r) st = rccl_status(r, r->CommDestroy(cm->c), "ncclCommDestroy");
  delete cm;
  return st;
}

static int allreduce_sum(void* comm, void* buf, int64_t n, ncclDataType_t dtype, void* stream, const char* who) {
  if (!comm || n < 0 || (n > 0 && !buf)) {
    set_error(std::string(who) + ": NULL comm / buffer or negative count");
    return GSLM_ERR_INVALID;
  }
  if (n == 0) return GSLM_OK;
  const Rccl* r = rccl();
  if (!r) return GSLM_ERR_HIP;
  Comm* cm = static_cast<Comm*>(comm);
  return rccl_status(r, r->AllReduce(buf, buf, (size_t)n, dtype, ncclSum, cm->c, (hipStream_t)stream), who);
}

int gslm_allreduce_sum_f32(void* comm, float* buf, int64_t n, void* stream) {
  return allreduce_sum(comm, buf, n, ncclFloat32, stream, "allreduce_sum_f32");
}

int gslm_allreduce_sum_f64(void* comm, double* buf, int64_t n, void* stream) {
  return allreduce_sum(comm, buf, n, ncclFloat64, stream, "allreduce_sum_f64");
}

int gslm_alltoall(void* comm, const void* send, void* recv, int64_t bytes_per_rank, void* stream) {
  if (!comm || bytes_per_rank < 0 || (bytes_per_rank > 0 && (!send || !recv))) {
    set_error("alltoall: NULL comm / buffers or negative size");
    return GSLM_ERR_INVALID;
  }
  if (bytes_per_rank == 0) return GSLM_OK;
  const Rccl* r = rccl();
  if (!r) return GSLM_ERR_HIP;
  Comm* cm = static_cast<Comm*>(comm);
  return rccl_status(r, r->AllToAll(send, recv, (size_t)bytes_per_rank, ncclInt8, cm->c, (hipStream_t)stream),
                     "ncclAllToAll");
}

int gslm_allgather(void* comm, const void* send, void* recv, int64_t bytes_per_rank, void* stream) {
  if (!comm || bytes_per_rank < 0 || (bytes_per_rank > 0 && (!send || !recv))) {
    set_error("allgather: NULL comm / buffers or negative size");
    return GSLM_ERR_INVALID;
  }
  if (bytes_per_rank == 0) return GSLM_OK;
  const Rccl* r = rccl();
  if (!r) return GSLM_ERR_HIP;
  Comm* cm = static_cast<Comm*>(comm);
  return rccl_status(r, r->AllGather(send, recv, (size_t)bytes_per_rank, ncclInt8, cm->c, (hipStream_t)stream),
                     "ncclAllGather");
}

}  // extern "C"

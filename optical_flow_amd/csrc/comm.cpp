// Gradient all-reduce over RCCL behind the C ABI (SURVEY.md §8 b "of_comm_*", §8 e).
//
// The reference trains in one process (train.py:47-61, no collectives anywhere); the batch
// data parallelism of configs 4-5 is build-added (K14): every rank runs train_step on its own
// shard and the gradient arena is summed across ranks in buckets while the backward is still
// running (optical_flow_amd/dist.py), the 1/N average folded into the Adam launch.
//
// librccl is resolved at of_comm_get_unique_id / of_comm_init time with dlopen("librccl.so.1"):
// inside a PyTorch process that is the RCCL torch already mapped (same soname, one instance),
// standalone it is /opt/rocm's.  Loading liboflow itself therefore needs no RCCL, and a
// process that never calls of_comm_* never touches it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include "common.h"

using namespace oflow;

struct of_comm {
  ncclComm_t nccl;
  int nranks, rank, device;
  int nonblocking;   // made by of_comm_init_timeout with a deadline (ncclConfig_t.blocking = 0)
};

namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*);
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
  // optional (non-blocking init with a deadline); absent in old RCCL builds
  ncclResult_t (*comm_init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*);
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t);
  ncclResult_t (*comm_destroy)(ncclComm_t);
  ncclResult_t (*comm_abort)(ncclComm_t);
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*);
  const char* (*error_string)(ncclResult_t);
  bool ok = false;
  std::string why;
};

RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      api.why = std::string("dlopen librccl.so.1: ") + dlerror();
      return;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
    api.get_unique_id = (decltype(api.get_unique_id))sym("ncclGetUniqueId");
    api.comm_init_rank = (decltype(api.comm_init_rank))sym("ncclCommInitRank");
    api.comm_init_rank_config =
        (decltype(api.comm_init_rank_config))sym("ncclCommInitRankConfig");
    api.all_reduce = (decltype(api.all_reduce))sym("ncclAllReduce");
    api.comm_destroy = (decltype(api.comm_destroy))sym("ncclCommDestroy");
    api.comm_abort = (decltype(api.comm_abort))sym("ncclCommAbort");
    api.async_error = (decltype(api.async_error))sym("ncclCommGetAsyncError");
    api.error_string = (decltype(api.error_string))sym("ncclGetErrorString");
    api.ok = api.get_unique_id && api.comm_init_rank && api.all_reduce && api.comm_destroy &&
             api.comm_abort && api.async_error && api.error_string;
    if (!api.ok) api.why = "librccl.so.1 lacks an nccl* entry point";
  });
  return api;
}

int rccl_fail(const char* what, ncclResult_t r) {
  return fail(OF_EHIP, std::string(what) + ": " + rccl().error_string(r));
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// A non-blocking communicator's state: poll until it leaves ncclInProgress or the deadline
// passes (deadline <= 0: no deadline).  Returns ncclSuccess, the failure, or ncclInProgress on
// expiry.
ncclResult_t settle(ncclComm_t c, double deadline) {
  for (;;) {
    ncclResult_t e = ncclSuccess;
    ncclResult_t r = rccl().async_error(c, &e);
    if (r != ncclSuccess) return r;
    if (e != ncclInProgress) return e;
    if (deadline > 0 && now_s() > deadline) return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

}  // namespace

extern "C" {

int of_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int of_comm_get_unique_id(void* id) {
  OF_CHECK_ARG(id, "comm_get_unique_id: id");
  RcclApi& api = rccl();
  if (!api.ok) return fail(OF_EUNSUPPORTED, api.why);
  ncclUniqueId u;
  ncclResult_t r = api.get_unique_id(&u);
  if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
  memcpy(id, &u, sizeof(u));
  return OF_OK;
}

int of_comm_probe(void) {
  RcclApi& api = rccl();
  if (!api.ok) return fail(OF_EUNSUPPORTED, api.why);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(OF_EHIP, "comm_probe: no current HIP device");
  return OF_OK;
}

int of_comm_init_timeout(of_comm** comm, const void* id, int nranks, int rank,
                         double timeout_s) {
  OF_CHECK_ARG(comm && id, "comm_init: comm, id");
  OF_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "comm_init: rank / nranks");
  *comm = nullptr;
  RcclApi& api = rccl();
  if (!api.ok) return fail(OF_EUNSUPPORTED, api.why);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(OF_EHIP, "comm_init: no current HIP device");
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  if (timeout_s > 0 && api.comm_init_rank_config) {
    // non-blocking: the call returns at once (ncclInProgress) and the rendezvous with the
    // other ranks completes in RCCL's own threads; a peer that never arrives leaves it in
    // progress, and at the deadline the half-made communicator is aborted
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const double deadline = now_s() + timeout_s;
    ncclResult_t r = api.comm_init_rank_config(&c, nranks, u, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (c) api.comm_abort(c);
      return rccl_fail("ncclCommInitRankConfig", r);
    }
    r = settle(c, deadline);
    if (r == ncclInProgress) {
      api.comm_abort(c);
      return fail(OF_ETIMEOUT, "ncclCommInitRankConfig: the " + std::to_string(nranks) +
                                   "-rank rendezvous did not complete within " +
                                   std::to_string(timeout_s) + " s (aborted)");
    }
    if (r != ncclSuccess) {
      api.comm_abort(c);
      return rccl_fail("ncclCommInitRankConfig", r);
    }
    *comm = new of_comm{c, nranks, rank, dev, 1};
    return OF_OK;
  }
  ncclResult_t r = api.comm_init_rank(&c, nranks, u, rank);   // collective over the ranks
  if (r != ncclSuccess) return rccl_fail("ncclCommInitRank", r);
  *comm = new of_comm{c, nranks, rank, dev, 0};
  return OF_OK;
}

int of_comm_init(of_comm** comm, const void* id, int nranks, int rank) {
  return of_comm_init_timeout(comm, id, nranks, rank, 0.0);
}

int of_comm_info(const of_comm* comm, int* nranks, int* rank, int* device) {
  OF_CHECK_ARG(comm, "comm_info: comm");
  if (nranks) *nranks = comm->nranks;
  if (rank) *rank = comm->rank;
  if (device) *device = comm->device;
  return OF_OK;
}

int of_comm_allreduce_ex_async(of_comm* comm, const float* send, float* recv, int64_t count,
                               int op, void* stream) {
  OF_CHECK_ARG(comm && send && recv && count >= 0, "comm_allreduce: args");
  OF_CHECK_ARG(op == OF_REDUCE_SUM || op == OF_REDUCE_AVG, "comm_allreduce: op");
  if (!comm->nccl) return fail(OF_EHIP, "comm_allreduce: the communicator was aborted");
  if (count == 0) return OF_OK;
  ncclResult_t r = rccl().all_reduce(send, recv, (size_t)count, ncclFloat32,
                                     op == OF_REDUCE_AVG ? ncclAvg : ncclSum, comm->nccl,
                                     as_stream(stream));
  // a non-blocking communicator may return while the enqueue is still in progress: it must
  // settle before the next call on the communicator (host-side only; the GPU work stays async)
  if (r == ncclInProgress && comm->nonblocking) r = settle(comm->nccl, 0.0);
  if (r != ncclSuccess) return rccl_fail("ncclAllReduce", r);
  return OF_OK;
}

int of_comm_allreduce_async(of_comm* comm, const float* send, float* recv, int64_t count,
                            void* stream) {
  return of_comm_allreduce_ex_async(comm, send, recv, count, OF_REDUCE_SUM, stream);
}

int of_comm_async_error(of_comm* comm) {
  OF_CHECK_ARG(comm, "comm_async_error: comm");
  if (!comm->nccl) return fail(OF_EHIP, "RCCL communicator: aborted");
  ncclResult_t e = ncclSuccess;
  ncclResult_t r = rccl().async_error(comm->nccl, &e);
  if (r != ncclSuccess) return rccl_fail("ncclCommGetAsyncError", r);
  if (e != ncclSuccess && e != ncclInProgress) return rccl_fail("RCCL communicator", e);
  return OF_OK;
}

int of_comm_abort(of_comm* comm) {
  OF_CHECK_ARG(comm, "comm_abort: comm");
  ncclComm_t c = comm->nccl;
  if (!c) return OF_OK;
  comm->nccl = nullptr;
  ncclResult_t r = rccl().comm_abort(c);
  if (r != ncclSuccess) return rccl_fail("ncclCommAbort", r);
  return OF_OK;
}

int of_comm_destroy(of_comm* comm, int abort) {
  if (!comm) return OF_OK;
  ncclResult_t r = ncclSuccess;
  if (comm->nccl) r = abort ? rccl().comm_abort(comm->nccl) : rccl().comm_destroy(comm->nccl);
  delete comm;
  if (r != ncclSuccess) return rccl_fail(abort ? "ncclCommAbort" : "ncclCommDestroy", r);
  return OF_OK;
}

}  // extern "C"

// Framework-owned RCCL communicator (host C++, links librccl + the HIP runtime).
//
// The reference has no collective code at all: distributed training is the user's
// NCCL.  polyaxon_amd uses torch.distributed (backend "nccl" = RCCL) for model DP, and this thin C++
// communicator for the framework's own collectives — cross-rank metric reduction inside DP trials, the
// HPO bracket-metric all-gather, and the xGMI bandwidth probe (rccl-tests all_reduce_perf equivalent) —
// without a Python/ProcessGroup layer in between.  Everything is enqueued on a caller-supplied hipStream_t
// so it overlaps compute and can be captured in a hipGraph.
//
//   plx_rccl_unique_id(out[128])                          rank 0 creates, ships via any side channel
//   plx_rccl_init(id, nranks, rank, device) -> handle (an integer id, never reused)
//   plx_rccl_all_reduce / all_gather / reduce_scatter / broadcast (dtype: 0 f32, 1 bf16, 2 f16, 3 f64, 4 i32)
//   plx_rccl_bus_bw(comm, bytes, iters, stream) -> measured algorithm + bus bandwidth of all-reduce
//   plx_rccl_destroy(comm)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <memory>
#include <unordered_map>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

ncclDataType_t dtype_of(int d) {
  switch (d) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclFloat64;
    default: return ncclInt32;
  }
}

ncclRedOp_t op_of(int o) {
  switch (o) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    default: return ncclAvg;
  }
}

struct Comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  ~Comm() {
    if (comm) ncclCommDestroy(comm);  // the last holder of a destroyed handle (see plx_rccl_destroy)
  }
};

// Live communicators by handle.  A handle is a monotonically increasing integer (never an address), so a destroyed
// handle can never alias a later communicator; every entry point takes a shared_ptr copy under the lock and runs its
// collective on that copy, so a plx_rccl_destroy on another thread cannot free the communicator mid-call: the
// ncclComm is destroyed when the last in-flight call drops its reference.
std::mutex g_mu;
std::unordered_map<uintptr_t, std::shared_ptr<Comm>> g_live;
uintptr_t g_next = 1;

std::shared_ptr<Comm> live(void* h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_live.find(reinterpret_cast<uintptr_t>(h));
  return it == g_live.end() ? nullptr : it->second;
}

}  // namespace

PLX_API int plx_rccl_unique_id(char* out) {
  static_assert(sizeof(ncclUniqueId) <= 128, "unique id too large");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  memset(out, 0, 128);
  memcpy(out, &id, sizeof(id));
  return 0;
}

PLX_API void* plx_rccl_init(const char* id_bytes, int nranks, int rank, int device, int* err) {
  if (hipSetDevice(device) != hipSuccess) {
    *err = -1;
    return nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  auto c = std::make_shared<Comm>();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
  if (r != ncclSuccess) {
    *err = (int)r;
    return nullptr;
  }
  c->comm = comm;
  *err = 0;
  std::lock_guard<std::mutex> lk(g_mu);
  const uintptr_t h = g_next++;
  g_live.emplace(h, std::move(c));
  return reinterpret_cast<void*>(h);
}

PLX_API int plx_rccl_all_reduce(void* h, const void* send, void* recv, int64_t count, int dtype, int op,
                                hipStream_t stream) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  return (int)ncclAllReduce(send, recv, (size_t)count, dtype_of(dtype), op_of(op), c->comm, stream);
}

PLX_API int plx_rccl_all_gather(void* h, const void* send, void* recv, int64_t count_per_rank, int dtype,
                                hipStream_t stream) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  return (int)ncclAllGather(send, recv, (size_t)count_per_rank, dtype_of(dtype), c->comm, stream);
}

PLX_API int plx_rccl_reduce_scatter(void* h, const void* send, void* recv, int64_t count_per_rank, int dtype, int op,
                                    hipStream_t stream) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  return (int)ncclReduceScatter(send, recv, (size_t)count_per_rank, dtype_of(dtype), op_of(op), c->comm, stream);
}

PLX_API int plx_rccl_broadcast(void* h, const void* send, void* recv, int64_t count, int dtype, int root,
                               hipStream_t stream) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  return (int)ncclBroadcast(send, recv, (size_t)count, dtype_of(dtype), root, c->comm, stream);
}

// All-reduce bandwidth probe on a device buffer of `bytes`: returns algbw and busbw (GB/s) like rccl-tests
// (busbw = algbw * 2 (n-1) / n).  Every collective's and HIP call's status is checked: a failing collective (or a
// destroyed communicator) returns its error code and reports no bandwidth.
PLX_API int plx_rccl_bus_bw(void* h, void* buf, int64_t bytes, int iters, hipStream_t stream, double* algbw,
                            double* busbw) {
  *algbw = *busbw = 0.0;
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  if (bytes < 4 || iters < 1) return (int)ncclInvalidArgument;
  const size_t count = (size_t)bytes / 4;
  for (int i = 0; i < 3; ++i) {
    const ncclResult_t r = ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, c->comm, stream);
    if (r != ncclSuccess) return (int)r;
  }
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess) return (int)ncclUnhandledCudaError;
  if (hipEventCreate(&b) != hipSuccess) {
    hipEventDestroy(a);
    return (int)ncclUnhandledCudaError;
  }
  int rc = 0;
  float ms = 0.f;
  if (hipEventRecord(a, stream) != hipSuccess) rc = (int)ncclUnhandledCudaError;
  for (int i = 0; i < iters && rc == 0; ++i) {
    const ncclResult_t r = ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, c->comm, stream);
    if (r != ncclSuccess) rc = (int)r;
  }
  if (rc == 0 && (hipEventRecord(b, stream) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
                  hipEventElapsedTime(&ms, a, b) != hipSuccess))
    rc = (int)ncclUnhandledCudaError;
  if (rc == 0) {  // an asynchronous failure of the enqueued collectives surfaces here
    ncclResult_t async = ncclSuccess;
    if (ncclCommGetAsyncError(c->comm, &async) != ncclSuccess || async != ncclSuccess)
      rc = (int)(async != ncclSuccess ? async : ncclInternalError);
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  if (rc) return rc;
  const double sec = ms / 1e3 / iters;
  *algbw = (double)bytes / sec / 1e9;
  *busbw = *algbw * 2.0 * (c->nranks - 1) / c->nranks;
  return 0;
}

PLX_API int plx_rccl_destroy(void* h) {
  std::shared_ptr<Comm> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_live.find(reinterpret_cast<uintptr_t>(h));
    if (it == g_live.end()) return h ? (int)ncclInvalidArgument : 0;
    c = std::move(it->second);
    g_live.erase(it);
  }
  if (c.use_count() > 1) return 0;  // a call in flight holds it: destroyed when that call returns (~Comm)
  const ncclResult_t r = ncclCommDestroy(c->comm);
  c->comm = nullptr;
  return (int)r;
}

PLX_API const char* plx_rccl_error(int code) { return ncclGetErrorString((ncclResult_t)code); }

// Framework-owned RCCL communicator with a watchdog (host C++, links librccl + the HIP runtime).
//
// The reference has no collective code at all: distributed training is the user's NCCL, and a failed
// rank is handled by tearing every rank of the experiment down (/root/reference/polyaxon/signals/experiments.py:252-281).
// polyaxon_amd runs every device collective of a DP trial on ONE communicator per process (parallel/comm.py): bucket
// all-reduces, ZeRO-1 reduce-scatter / all-gather, the parameter broadcast, the metric mean.  Everything is enqueued on
// a caller-supplied hipStream_t so it overlaps compute.
//
// Failure detection.  The communicator is created NON-BLOCKING (ncclCommInitRankConfig, blocking = 0)
// and its initialisation is polled with ncclCommGetAsyncError against a deadline: a peer that never joins aborts the
// communicator (ncclCommAbort) and fails plx_rccl_init with PLX_RCCL_TIMEOUT instead of blocking forever.  After init
// a per-process watchdog thread checks every live communicator every few ms:
//   * an asynchronous RCCL error (ncclCommGetAsyncError) aborts it;
//   * every enqueued collective records a completion event on its stream; a collective still incomplete after the
//     communicator's timeout (a peer stuck in a kernel, a peer that stopped issuing collectives) aborts it.
// ncclCommAbort makes the RCCL kernels in flight exit, so a host thread blocked on the stream returns; every later call
// on the communicator returns the recorded error (Python: RcclError), the rank's process fails, and polyflow tears the
// gang down (polyflow/scheduler.py).
//
//   plx_rccl_unique_id(out[128])                          rank 0 creates, ships via any side channel
//   plx_rccl_init(id, nranks, rank, device, init_timeout_ms, coll_timeout_ms, err) -> handle (integer id, never reused)
//   plx_rccl_all_reduce / all_gather / reduce_scatter / broadcast (dtype: 0 f32, 1 bf16, 2 f16, 3 f64, 4 i32)
//   plx_rccl_status(comm)        0, or the error that aborted it
//   plx_rccl_bus_bw(comm, bytes, iters, stream) -> measured algorithm + bus bandwidth of all-reduce
//   plx_rccl_destroy(comm)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kTimeout = 1000;  // PLX_RCCL_TIMEOUT: the watchdog aborted the communicator on a deadline
constexpr int kAborted = 1001;  // the communicator was aborted (plx_rccl_abort)

using Clock = std::chrono::steady_clock;

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

struct Pending {
  hipEvent_t ev;
  Clock::time_point t0;
};

struct Comm {
  std::mutex mu;                  // guards comm (enqueue vs abort), pending, free_events
  ncclComm_t comm = nullptr;      // nullptr once aborted or destroyed
  std::atomic<int> error{0};      // sticky: the error that aborted the communicator
  int nranks = 0, rank = 0, device = 0;
  int64_t timeout_ms = 0;         // collective deadline (0: no progress watchdog, async errors still abort)
  std::deque<Pending> pending;    // collectives enqueued, oldest first
  std::vector<hipEvent_t> free_events;

  // caller holds mu
  void abort_locked(int why) {
    int expect = 0;
    error.compare_exchange_strong(expect, why);
    if (comm) {
      ncclCommAbort(comm);        // RCCL kernels in flight observe the abort flag and exit
      comm = nullptr;
    }
  }

  ~Comm() {
    for (auto& p : pending) hipEventDestroy(p.ev);
    for (auto e : free_events) hipEventDestroy(e);
    if (comm) ncclCommDestroy(comm);  // the last holder of a destroyed handle (see plx_rccl_destroy)
  }
};

// Live communicators by handle.  A handle is a monotonically increasing integer (never an address), so a destroyed
// handle can never alias a later communicator; every entry point takes a shared_ptr copy under the lock and runs its
// collective on that copy, so a plx_rccl_destroy on another thread cannot free the communicator mid-call.
// (leaked on purpose: the detached watchdog thread may still read them while the process exits)
std::mutex& g_mu = *new std::mutex;
std::unordered_map<uintptr_t, std::shared_ptr<Comm>>& g_live = *new std::unordered_map<uintptr_t, std::shared_ptr<Comm>>;
uintptr_t g_next = 1;

std::shared_ptr<Comm> live(void* h) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_live.find(reinterpret_cast<uintptr_t>(h));
  return it == g_live.end() ? nullptr : it->second;
}

// ---- watchdog: one thread per process, started with the first communicator that has a deadline or needs async
// error polling; it sleeps while no communicator is live
std::mutex& g_wd_mu = *new std::mutex;
std::mutex& g_pass_mu = *new std::mutex;  // held for a whole pass: exit waits for the pass in progress
std::condition_variable& g_wd_cv = *new std::condition_variable;
bool g_wd_started = false;
std::atomic<bool> g_wd_stop{false};
constexpr int64_t kWdPeriodMs = 20;

void watchdog_pass() {
  std::vector<std::shared_ptr<Comm>> comms;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    comms.reserve(g_live.size());
    for (auto& kv : g_live) comms.push_back(kv.second);
  }
  const auto now = Clock::now();
  for (auto& c : comms) {
    std::unique_lock<std::mutex> lk(c->mu, std::try_to_lock);
    if (!lk.owns_lock() || !c->comm) continue;  // an enqueue in progress: next pass
    ncclResult_t async = ncclSuccess;
    if (ncclCommGetAsyncError(c->comm, &async) == ncclSuccess && async != ncclSuccess && async != ncclInProgress) {
      c->abort_locked((int)async);
      continue;
    }
    // retire completed collectives in order; the oldest incomplete one decides the deadline
    while (!c->pending.empty()) {
      Pending& p = c->pending.front();
      const hipError_t q = hipEventQuery(p.ev);
      if (q == hipErrorNotReady) break;
      c->free_events.push_back(p.ev);
      c->pending.pop_front();
    }
    if (c->timeout_ms > 0 && !c->pending.empty()) {
      const auto age = std::chrono::duration_cast<std::chrono::milliseconds>(now - c->pending.front().t0).count();
      if (age > c->timeout_ms) c->abort_locked(kTimeout);
    }
  }
}

void watchdog_main() {
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(g_wd_mu);
      g_wd_cv.wait_for(lk, std::chrono::milliseconds(kWdPeriodMs));
    }
    std::lock_guard<std::mutex> pass(g_pass_mu);
    if (g_wd_stop.load()) return;
    watchdog_pass();
  }
}

// atexit (registered after the HIP runtime initialised, so it runs before the runtime's own teardown): stop the
// watchdog and wait for a pass in progress, so no HIP / RCCL call races the process exit
void stop_watchdog() {
  g_wd_stop.store(true);
  std::lock_guard<std::mutex> pass(g_pass_mu);
}

void ensure_watchdog() {
  std::lock_guard<std::mutex> lk(g_wd_mu);
  if (g_wd_started) return;
  g_wd_started = true;
  atexit(stop_watchdog);
  std::thread(watchdog_main).detach();
}

// Non-blocking communicator calls may return ncclInProgress: poll until the call completed, failed or the deadline
// passed (caller holds c->mu).  Returns 0 or an error code.
int settle_locked(Comm* c, ncclResult_t r, int64_t deadline_ms) {
  if (r != ncclSuccess && r != ncclInProgress) return (int)r;
  const auto t0 = Clock::now();
  for (;;) {
    ncclResult_t async = ncclSuccess;
    if (ncclCommGetAsyncError(c->comm, &async) != ncclSuccess) return (int)ncclInternalError;
    if (async == ncclSuccess) return 0;
    if (async != ncclInProgress) return (int)async;
    if (deadline_ms > 0 &&
        std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() > deadline_ms)
      return kTimeout;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// Enqueue one collective: refuse on an aborted communicator, settle an in-progress return, record the completion
// event the watchdog retires (skipped while the stream is being captured into a graph: a captured event cannot be
// queried)
template <typename F>
int enqueue(void* h, hipStream_t stream, F&& call) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->error.load()) return c->error.load();
  if (!c->comm) return (int)ncclInvalidArgument;
  int rc = settle_locked(c.get(), call(c->comm), c->timeout_ms);
  if (rc) {
    c->abort_locked(rc);
    return rc;
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return 0;
  hipEvent_t ev = nullptr;
  if (!c->free_events.empty()) {
    ev = c->free_events.back();
    c->free_events.pop_back();
  } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    return 0;  // no event: this collective is not tracked (async errors still are)
  }
  if (hipEventRecord(ev, stream) != hipSuccess) {
    c->free_events.push_back(ev);
    return 0;
  }
  c->pending.push_back({ev, Clock::now()});
  return 0;
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

// init_timeout_ms: deadline for every rank to join (0: none); coll_timeout_ms: per-collective deadline of the
// watchdog (0: none -- asynchronous RCCL errors still abort)
PLX_API void* plx_rccl_init(const char* id_bytes, int nranks, int rank, int device, int64_t init_timeout_ms,
                            int64_t coll_timeout_ms, int* err) {
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
  c->timeout_ms = coll_timeout_ms > 0 ? coll_timeout_ms : 0;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t comm = nullptr;
  const ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (comm) ncclCommAbort(comm);
    *err = (int)r;
    return nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(c->mu);
    c->comm = comm;
    const int rc = settle_locked(c.get(), r, init_timeout_ms);
    if (rc) {
      c->abort_locked(rc);
      *err = rc;
      return nullptr;
    }
  }
  *err = 0;
  ensure_watchdog();
  std::lock_guard<std::mutex> lk(g_mu);
  const uintptr_t h = g_next++;
  g_live.emplace(h, std::move(c));
  return reinterpret_cast<void*>(h);
}

PLX_API int plx_rccl_all_reduce(void* h, const void* send, void* recv, int64_t count, int dtype, int op,
                                hipStream_t stream) {
  return enqueue(h, stream, [&](ncclComm_t comm) {
    return ncclAllReduce(send, recv, (size_t)count, dtype_of(dtype), op_of(op), comm, stream);
  });
}

PLX_API int plx_rccl_all_gather(void* h, const void* send, void* recv, int64_t count_per_rank, int dtype,
                                hipStream_t stream) {
  return enqueue(h, stream, [&](ncclComm_t comm) {
    return ncclAllGather(send, recv, (size_t)count_per_rank, dtype_of(dtype), comm, stream);
  });
}

PLX_API int plx_rccl_reduce_scatter(void* h, const void* send, void* recv, int64_t count_per_rank, int dtype, int op,
                                    hipStream_t stream) {
  return enqueue(h, stream, [&](ncclComm_t comm) {
    return ncclReduceScatter(send, recv, (size_t)count_per_rank, dtype_of(dtype), op_of(op), comm, stream);
  });
}

PLX_API int plx_rccl_broadcast(void* h, const void* send, void* recv, int64_t count, int dtype, int root,
                               hipStream_t stream) {
  return enqueue(h, stream, [&](ncclComm_t comm) {
    return ncclBroadcast(send, recv, (size_t)count, dtype_of(dtype), root, comm, stream);
  });
}

// 0 while healthy, else the error that aborted the communicator (PLX_RCCL_TIMEOUT, an RCCL error code, ...)
PLX_API int plx_rccl_status(void* h) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  return c->error.load();
}

// collectives enqueued and not yet seen complete by the watchdog (tests)
PLX_API int plx_rccl_pending(void* h) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return -1;
  std::lock_guard<std::mutex> lk(c->mu);
  return (int)c->pending.size();
}

PLX_API int plx_rccl_set_timeout(void* h, int64_t coll_timeout_ms) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(c->mu);
  c->timeout_ms = coll_timeout_ms > 0 ? coll_timeout_ms : 0;
  return 0;
}

// abort now (a rank that knows its gang failed): in-flight RCCL kernels exit, later calls return kAborted
PLX_API int plx_rccl_abort(void* h) {
  const std::shared_ptr<Comm> c = live(h);
  if (!c) return (int)ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(c->mu);
  c->abort_locked(kAborted);
  return 0;
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
  const int64_t count = bytes / 4;
  for (int i = 0; i < 3; ++i) {
    const int r = plx_rccl_all_reduce(h, buf, buf, count, 0, 0, stream);
    if (r) return r;
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
  for (int i = 0; i < iters && rc == 0; ++i) rc = plx_rccl_all_reduce(h, buf, buf, count, 0, 0, stream);
  if (rc == 0 && (hipEventRecord(b, stream) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
                  hipEventElapsedTime(&ms, a, b) != hipSuccess))
    rc = (int)ncclUnhandledCudaError;
  if (rc == 0) rc = c->error.load();  // an asynchronous failure (the watchdog aborted it) surfaces here
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
  if (c.use_count() > 1) return 0;  // a call in flight (or the watchdog) holds it: destroyed with the last reference
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->comm) return 0;           // aborted: ncclCommAbort already freed it
  ncclResult_t r = ncclCommFinalize(c->comm);
  if (r == ncclSuccess || r == ncclInProgress) r = (ncclResult_t)settle_locked(c.get(), r, c->timeout_ms);
  if (r != ncclSuccess) {
    ncclCommAbort(c->comm);         // a finalize that cannot complete (a dead peer): abort instead of hanging
    c->comm = nullptr;
    return (int)r;
  }
  r = ncclCommDestroy(c->comm);
  c->comm = nullptr;
  return (int)r;
}

PLX_API const char* plx_rccl_error(int code) {
  if (code == kTimeout) return "timed out (the watchdog aborted the communicator: a peer did not join or progress)";
  if (code == kAborted) return "communicator aborted";
  if (code == -1) return "hipSetDevice failed";
  return ncclGetErrorString((ncclResult_t)code);
}

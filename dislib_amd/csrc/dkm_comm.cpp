// dkm_comm.cpp -- the one collective of the Lloyd iteration: an in-place
// RCCL all-reduce (sum) of each GPU's packed [sums k*d | counts k] fp64
// buffer over xGMI.  Replaces the reference's `_merge` arity tree and the
// `compss_wait_on` gather (dislib/cluster/kmeans/base.py:137-143, 184-191):
// after it every rank holds the global sums, runs the same centre update and
// reaches the same convergence decision -- no broadcast of centres.
//
// librccl is resolved at the first call (dlopen, not a link-time
// dependency): an RCCL already mapped into the process (PyTorch's, for a
// process that also runs torch.distributed) is reused -- RTLD_NOLOAD -- so
// one process never carries two RCCL builds; otherwise ROCm's own.
//
// Communicators are kept per device:
//   one process per GPU (torchrun): dkm_allreduce_unique_id on rank 0, the
//     128-byte id handed to every rank by the caller, then
//     dkm_allreduce_init_rank on every rank;
//   one process driving several GPUs: dkm_allreduce_init(ndev, devs).
// dkm_allreduce_sum_f64(buf, count, device, stream) then reduces on the
// communicator of `device`, stream-ordered.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "../../include/dkm.h"

namespace dkm {
int fail(int code, const std::string &msg);
}

namespace {

struct Rccl {
  void *h = nullptr;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
};

std::mutex g_mu;
Rccl g_r;
std::map<int, ncclComm_t> g_comms;  // device -> communicator

int load_rccl() {
  if (g_r.h) return 0;
  const char *names[] = {"librccl.so", "librccl.so.1"};
  void *h = nullptr;
  for (const char *n : names)
    if ((h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;
  for (const char *n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
    if (!h && (h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
  if (!h)
    return dkm::fail(DKM_E_COMM, std::string("librccl not found: ") + dlerror());
  Rccl r;
  r.h = h;
  r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
  r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
  r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
  r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
  r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
  r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
  r.count = (decltype(r.count))dlsym(h, "ncclCommCount");
  r.user_rank = (decltype(r.user_rank))dlsym(h, "ncclCommUserRank");
  if (!r.get_id || !r.init_rank || !r.init_all || !r.all_reduce ||
      !r.destroy || !r.err || !r.count || !r.user_rank)
    return dkm::fail(DKM_E_COMM, "librccl lacks an nccl entry point");
  g_r = r;
  return 0;
}

int rccl_fail(const char *what, ncclResult_t rc) {
  return dkm::fail(DKM_E_COMM, std::string(what) + ": " + g_r.err(rc));
}

// run f with `device` current, restoring the caller's device
template <class F>
int on_device(int device, F &&f) {
  int old = -1;
  if (hipGetDevice(&old) != hipSuccess) old = -1;
  if (hipSetDevice(device) != hipSuccess)
    return dkm::fail(DKM_E_ARG, "allreduce: bad device " + std::to_string(device));
  const int r = f();
  if (old >= 0) (void)hipSetDevice(old);
  return r;
}

}  // namespace

extern "C" {

int dkm_allreduce_unique_id(void *id) {
  if (!id) return dkm::fail(DKM_E_ARG, "allreduce_unique_id: NULL");
  std::lock_guard<std::mutex> lk(g_mu);
  if (int r = load_rccl()) return r;
  ncclUniqueId u;
  if (ncclResult_t rc = g_r.get_id(&u)) return rccl_fail("ncclGetUniqueId", rc);
  memcpy(id, &u, sizeof(u));
  return 0;
}

int dkm_allreduce_init_rank(const void *id, int nranks, int rank, int device) {
  if (!id || nranks < 1 || rank < 0 || rank >= nranks || device < 0)
    return dkm::fail(DKM_E_ARG, "allreduce_init_rank: bad arguments");
  std::lock_guard<std::mutex> lk(g_mu);
  if (int r = load_rccl()) return r;
  if (g_comms.count(device))
    return dkm::fail(DKM_E_ARG, "allreduce_init_rank: device already has a "
                                "communicator (dkm_allreduce_finalize first)");
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  return on_device(device, [&]() -> int {
    ncclComm_t c = nullptr;
    if (ncclResult_t rc = g_r.init_rank(&c, nranks, u, rank))
      return rccl_fail("ncclCommInitRank", rc);
    g_comms[device] = c;
    return 0;
  });
}

int dkm_allreduce_init(int ndev, const int *devs) {
  if (ndev < 1 || !devs) return dkm::fail(DKM_E_ARG, "allreduce_init: bad arguments");
  std::lock_guard<std::mutex> lk(g_mu);
  if (int r = load_rccl()) return r;
  for (int i = 0; i < ndev; ++i)
    if (devs[i] < 0 || g_comms.count(devs[i]))
      return dkm::fail(DKM_E_ARG, "allreduce_init: bad or already initialised "
                                  "device " + std::to_string(devs[i]));
  ncclComm_t *c = new ncclComm_t[ndev];
  int old = -1;
  if (hipGetDevice(&old) != hipSuccess) old = -1;
  const ncclResult_t rc = g_r.init_all(c, ndev, devs);
  if (old >= 0) (void)hipSetDevice(old);
  if (rc) {
    delete[] c;
    return rccl_fail("ncclCommInitAll", rc);
  }
  for (int i = 0; i < ndev; ++i) g_comms[devs[i]] = c[i];
  delete[] c;
  return 0;
}

int dkm_allreduce_sum_f64(double *buf, int64_t count, int device,
                          void *stream) {
  if (count < 0 || (count > 0 && !buf))
    return dkm::fail(DKM_E_ARG, "allreduce_sum_f64: bad buffer");
  ncclComm_t c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(device);
    if (it == g_comms.end())
      return dkm::fail(DKM_E_ARG, "allreduce_sum_f64: no communicator on device " +
                                      std::to_string(device));
    c = it->second;
  }
  if (count == 0) return 0;
  if (ncclResult_t rc = g_r.all_reduce(buf, buf, (size_t)count, ncclFloat64,
                                       ncclSum, c, (hipStream_t)stream))
    return rccl_fail("ncclAllReduce", rc);
  return 0;
}

int dkm_allreduce_finalize(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  int r = 0;
  for (auto &kv : g_comms) {
    if (ncclResult_t rc = g_r.destroy(kv.second)) r = rccl_fail("ncclCommDestroy", rc);
  }
  g_comms.clear();
  return r;
}

int dkm_allreduce_finalize_device(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_comms.find(device);
  if (it == g_comms.end()) return 0;
  const ncclResult_t rc = g_r.destroy(it->second);
  g_comms.erase(it);
  return rc ? rccl_fail("ncclCommDestroy", rc) : 0;
}

int dkm_allreduce_available(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return load_rccl();
}

int dkm_allreduce_comm_info(int device, int *nranks, int *rank) {
  if (!nranks || !rank) return dkm::fail(DKM_E_ARG, "allreduce_comm_info: NULL");
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_comms.find(device);
  if (it == g_comms.end())
    return dkm::fail(DKM_E_ARG, "allreduce_comm_info: no communicator on "
                                "device " + std::to_string(device));
  if (ncclResult_t rc = g_r.count(it->second, nranks))
    return rccl_fail("ncclCommCount", rc);
  if (ncclResult_t rc = g_r.user_rank(it->second, rank))
    return rccl_fail("ncclCommUserRank", rc);
  return 0;
}

}  // extern "C"

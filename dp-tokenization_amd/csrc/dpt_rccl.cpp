// dpt_rccl.cpp -- the histogram all-reduce of a sharded corpus through RCCL, without torch (ABI 6).
//
// SURVEY.md §8(b) names `dpt_hist_allreduce(int64_t*, size_t, void* rccl_comm, void* stream)` and §8(e)
// one process per GPU over "torch.distributed (RCCL backend) or direct RCCL with a file-store unique
// id".  bench.py takes the torch route (dptok/dist.py); these four entry points are the direct one, for a
// caller that binds only the C-ABI.  The reference itself is single-process (llama_s2orc.sh:10), so no
// reference call site exists: the layout summed is dpt_token_histogram's (dpt_api.cpp).
//
// RCCL is resolved on first use with dlopen("librccl.so.1"): in a process that already holds an RCCL
// (PyTorch-ROCm ships one under the same SONAME) the loader returns that copy, so one communicator
// world is not split over two libraries; libdpt.so has no link-time dependency on RCCL.  Only the
// header's types are used here.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <string>

#include "../../include/dpt.h"

static_assert(sizeof(ncclUniqueId) == DPT_RCCL_ID_BYTES, "ncclUniqueId size");

namespace dpt {
void set_last_error(const std::string &msg);   // dpt_api.cpp
}

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) err_str = nullptr;
    std::string load_error;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char *e = dlerror();
            r.load_error = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
            return;
        }
        r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
        r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.err_str = (decltype(r.err_str))dlsym(h, "ncclGetErrorString");
        if (!r.get_id || !r.init_rank || !r.destroy || !r.all_reduce || !r.err_str) {
            r.get_id = nullptr;
            r.load_error = "librccl.so.1 lacks an nccl* entry point";
        }
    });
    return r;
}

int rfail(const std::string &msg) {
    dpt::set_last_error(msg);
    return DPT_E_RCCL;
}

int rcheck(const Rccl &r, ncclResult_t res, const char *what) {
    if (res == ncclSuccess) return DPT_OK;
    return rfail(std::string(what) + ": " + r.err_str(res));
}

}  // namespace

extern "C" {

int dpt_rccl_get_unique_id(uint8_t *id_out) {
    if (!id_out) {
        dpt::set_last_error("null id_out");
        return DPT_E_ARG;
    }
    const Rccl &r = rccl();
    if (!r.get_id) return rfail(r.load_error);
    ncclUniqueId id;
    const int rc = rcheck(r, r.get_id(&id), "ncclGetUniqueId");
    if (rc == DPT_OK) memcpy(id_out, &id, sizeof id);
    return rc;
}

int dpt_rccl_comm_create(const uint8_t *id, int world, int rank, int device, void **comm_out) {
    if (!id || !comm_out || world < 1 || rank < 0 || rank >= world || device < 0) {
        dpt::set_last_error("bad communicator arguments (id, comm_out non-null; 0 <= rank < world; device >= 0)");
        return DPT_E_ARG;
    }
    *comm_out = nullptr;
    const Rccl &r = rccl();
    if (!r.get_id) return rfail(r.load_error);
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) {
        dpt::set_last_error(std::string("hipSetDevice: ") + hipGetErrorString(he));
        return DPT_E_HIP;
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    ncclComm_t comm = nullptr;
    const int rc = rcheck(r, r.init_rank(&comm, world, uid, rank), "ncclCommInitRank");   // (bound to `device`)
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    if (rc == DPT_OK) *comm_out = comm;
    return rc;
}

int dpt_rccl_comm_destroy(void *rccl_comm) {
    if (!rccl_comm) return DPT_OK;
    const Rccl &r = rccl();
    if (!r.get_id) return rfail(r.load_error);
    return rcheck(r, r.destroy((ncclComm_t)rccl_comm), "ncclCommDestroy");
}

int dpt_hist_allreduce(int64_t *hist, size_t n, void *rccl_comm, void *hip_stream) {
    if (!hist || !rccl_comm) {
        dpt::set_last_error("null hist or rccl_comm");
        return DPT_E_ARG;
    }
    if (!n) return DPT_OK;
    const Rccl &r = rccl();
    if (!r.get_id) return rfail(r.load_error);
    return rcheck(r, r.all_reduce(hist, hist, n, ncclInt64, ncclSum, (ncclComm_t)rccl_comm, (hipStream_t)hip_stream),
                  "ncclAllReduce");
}

}  // extern "C"

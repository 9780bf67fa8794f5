// comm.cpp -- the multi-GPU exchange behind the C ABI: RCCL over xGMI.
//
// Frames shard by global index with no data-path collective; what crosses
// GPUs is ONE all-reduce of the [points x 7] int64 counter matrix per
// Monte-Carlo step (the reference's parent-side sum of its workers' block
// results, python_ldpc_app/main.py:149-175), plus the bench's barrier and
// max-over-ranks of its wall clock.  librccl.so.1 is dlopen'ed on first use:
// single-GPU users never map its ~570 MB.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "ldpc_internal.h"

namespace {

struct Rccl {
    void *h = nullptr;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
};

std::mutex g_mu;
Rccl g_rccl;

// Load librccl once; returns nullptr (message in ldpc_last_error) if absent.
const Rccl *rccl() {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_rccl.h) return &g_rccl;
    const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    void *h = nullptr;
    for (const char *n : names)
        if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) {
        ldpc_fail(LDPC_EDEVICE, "RCCL not available: dlopen(librccl.so.1) failed: %s", dlerror());
        return nullptr;
    }
    Rccl r;
    r.h = h;
    r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
    r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
    if (!r.get_id || !r.init_rank || !r.all_reduce || !r.destroy || !r.err) {
        dlclose(h);
        ldpc_fail(LDPC_EDEVICE, "librccl.so.1 lacks an nccl* entry point");
        return nullptr;
    }
    g_rccl = r;
    return &g_rccl;
}

int nccl_fail(const Rccl *r, ncclResult_t e, const char *what) {
    return ldpc_fail(LDPC_EDEVICE, "%s failed: %s", what, r->err ? r->err(e) : "?");
}

}  // namespace

struct ldpc_comm {
    const Rccl *r = nullptr;
    ncclComm_t comm = nullptr;
    int device = 0, rank = 0, world = 1;
    hipStream_t stream = nullptr;  // for host-buffer reductions
    void *scratch = nullptr;       // device staging of host buffers
    size_t scratch_bytes = 0;
};

extern "C" {

int ldpc_comm_unique_id(uint8_t *id_out) {
    if (!id_out) return ldpc_fail(LDPC_EINVAL, "ldpc_comm_unique_id: NULL output");
    const Rccl *r = rccl();
    if (!r) return LDPC_EDEVICE;
    ncclUniqueId id;
    if (ncclResult_t e = r->get_id(&id)) return nccl_fail(r, e, "ncclGetUniqueId");
    static_assert(sizeof(id) == LDPC_COMM_ID_BYTES, "unique id size");
    std::memcpy(id_out, &id, sizeof(id));
    return LDPC_OK;
}

int ldpc_comm_init(const uint8_t *id, int32_t rank, int32_t world, int32_t device, ldpc_comm **out) {
    if (!out) return ldpc_fail(LDPC_EINVAL, "ldpc_comm_init: out is NULL");
    *out = nullptr;
    if (!id || world < 1 || rank < 0 || rank >= world || device < 0)
        return ldpc_fail(LDPC_EINVAL, "ldpc_comm_init: bad arguments (rank %d world %d device %d)", rank, world,
                         device);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev)
        return ldpc_fail(LDPC_EDEVICE, "ldpc_comm_init: device %d not visible (%d devices)", device, ndev);
    const Rccl *r = rccl();
    if (!r) return LDPC_EDEVICE;
    DeviceGuard dg(device);  // the caller's current device is restored on return
    auto *c = new ldpc_comm;
    c->r = r;
    c->device = device;
    c->rank = rank;
    c->world = world;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    if (ncclResult_t e = r->init_rank(&c->comm, world, uid, rank)) {
        delete c;
        return nccl_fail(r, e, "ncclCommInitRank");
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        (void)r->destroy(c->comm);
        delete c;
        return ldpc_fail(LDPC_EDEVICE, "ldpc_comm_init: hipStreamCreate failed");
    }
    *out = c;
    return LDPC_OK;
}

int ldpc_comm_allreduce(ldpc_comm *c, void *buf, int64_t count, int32_t dtype, int32_t op, uint32_t flags,
                        void *stream) {
    if (!c) return ldpc_fail(LDPC_EINVAL, "ldpc_comm_allreduce: NULL communicator");
    if (count < 0 || (count > 0 && !buf) || (dtype != LDPC_DT_I64 && dtype != LDPC_DT_F64) ||
        (op != LDPC_OP_SUM && op != LDPC_OP_MAX))
        return ldpc_fail(LDPC_EINVAL, "ldpc_comm_allreduce: bad arguments");
    if (count == 0) return LDPC_OK;
    DeviceGuard dg(c->device);
    const ncclDataType_t dt = dtype == LDPC_DT_I64 ? ncclInt64 : ncclFloat64;
    const ncclRedOp_t ro = op == LDPC_OP_SUM ? ncclSum : ncclMax;
    const size_t bytes = (size_t)count * 8;
    if (flags & LDPC_F_DEVICE_PTRS) {
        if (ncclResult_t e = c->r->all_reduce(buf, buf, (size_t)count, dt, ro, c->comm, (hipStream_t)stream))
            return nccl_fail(c->r, e, "ncclAllReduce");
        return LDPC_OK;
    }
    if (c->scratch_bytes < bytes) {
        (void)hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_bytes = 0;
        if (hipMalloc(&c->scratch, bytes) != hipSuccess)
            return ldpc_fail(LDPC_ENOMEM, "ldpc_comm_allreduce: hipMalloc(%zu) failed", bytes);
        c->scratch_bytes = bytes;
    }
    hipStream_t s = c->stream;
    if (hipMemcpyAsync(c->scratch, buf, bytes, hipMemcpyHostToDevice, s) != hipSuccess)
        return ldpc_fail(LDPC_EDEVICE, "ldpc_comm_allreduce: upload failed");
    if (ncclResult_t e = c->r->all_reduce(c->scratch, c->scratch, (size_t)count, dt, ro, c->comm, s))
        return nccl_fail(c->r, e, "ncclAllReduce");
    if (hipMemcpyAsync(buf, c->scratch, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return ldpc_fail(LDPC_EDEVICE, "ldpc_comm_allreduce: download failed");
    return LDPC_OK;
}

int ldpc_comm_barrier(ldpc_comm *c) {
    if (!c) return ldpc_fail(LDPC_EINVAL, "ldpc_comm_barrier: NULL communicator");
    int64_t one = 1;
    if (int rc = ldpc_comm_allreduce(c, &one, 1, LDPC_DT_I64, LDPC_OP_SUM, 0, nullptr)) return rc;
    if (one != c->world) return ldpc_fail(LDPC_EDEVICE, "ldpc_comm_barrier: %lld of %d ranks", (long long)one, c->world);
    return ldpc_device_synchronize(c->device);
}

int ldpc_comm_destroy(ldpc_comm *c) {
    if (!c) return LDPC_OK;
    DeviceGuard dg(c->device);
    if (c->comm) (void)c->r->destroy(c->comm);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    (void)hipFree(c->scratch);
    delete c;
    return LDPC_OK;
}

int ldpc_device_synchronize(int32_t device) {
    int ndev = 0;
    if (device < 0 || hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev)
        return ldpc_fail(LDPC_EDEVICE, "ldpc_device_synchronize: device %d not visible", device);
    DeviceGuard dg(device);
    if (hipDeviceSynchronize() != hipSuccess)
        return ldpc_fail(LDPC_EDEVICE, "ldpc_device_synchronize(%d) failed", device);
    return LDPC_OK;
}

}  // extern "C"

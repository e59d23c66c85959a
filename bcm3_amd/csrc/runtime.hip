// runtime.hip -- the device runtime the C++ host sampler (csrc/host/SamplerPTDevice.cpp) drives
// through the C-ABI: device memory, streams, and the point-to-point transport of the PT swap
// between neighbouring ranks over RCCL (xGMI between the GPUs of a node). Keeps every HIP / RCCL
// call in this hipcc-built library; libbcm3.so stays plain C++ on top of include/bcm3hip.h.
//
// The PT swap is the only cross-GPU traffic of the sampler: per exchange round,
// one {values[d], llh, lprior, lpp, T} record each way between ring neighbours (SamplerPT.cpp:
// 277-306 with the ladder sliced over ranks), grouped into one ncclGroupStart/End.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>

#include "../../include/bcm3hip.h"

static_assert(sizeof(ncclUniqueId) <= BCM3HIP_NCCL_ID_BYTES, "ncclUniqueId larger than the C-ABI buffer");

extern "C" {

int bcm3hip_set_device(int device) { return hipSetDevice(device) == hipSuccess ? 0 : BCM3HIP_ERR_HIP; }

int bcm3hip_malloc(void** ptr, size_t bytes)
{
    if (!ptr) return BCM3HIP_ERR_ARG;
    *ptr = nullptr;
    if (bytes == 0) return 0;
    if (hipMalloc(ptr, bytes) != hipSuccess) return BCM3HIP_ERR_ALLOC;
    return 0;
}

int bcm3hip_free(void* ptr) { return (!ptr || hipFree(ptr) == hipSuccess) ? 0 : BCM3HIP_ERR_HIP; }

int bcm3hip_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream)
{
    if (bytes == 0) return 0;
    if (!dst || !src) return BCM3HIP_ERR_ARG;
    const hipMemcpyKind k = kind == BCM3HIP_H2D ? hipMemcpyHostToDevice
                            : kind == BCM3HIP_D2H ? hipMemcpyDeviceToHost
                                                  : hipMemcpyDeviceToDevice;
    return hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream) == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_memset_async(void* dst, int value, size_t bytes, void* stream)
{
    if (bytes == 0) return 0;
    if (!dst) return BCM3HIP_ERR_ARG;
    return hipMemsetAsync(dst, value, bytes, (hipStream_t)stream) == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_stream_create(void** stream)
{
    if (!stream) return BCM3HIP_ERR_ARG;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return BCM3HIP_ERR_HIP;
    *stream = s;
    return 0;
}

int bcm3hip_stream_destroy(void* stream)
{
    return (!stream || hipStreamDestroy((hipStream_t)stream) == hipSuccess) ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_stream_synchronize(void* stream)
{
    return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

// ---- RCCL transport ----

int bcm3hip_nccl_get_unique_id(void* id)
{
    if (!id) return BCM3HIP_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return BCM3HIP_ERR_HIP;
    std::memset(id, 0, BCM3HIP_NCCL_ID_BYTES);
    std::memcpy(id, &u, sizeof(u));
    return 0;
}

int bcm3hip_nccl_comm_init(const void* id, int rank, int world, void** comm)
{
    if (!id || !comm || world < 1 || rank < 0 || rank >= world) return BCM3HIP_ERR_ARG;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t c;
    if (ncclCommInitRank(&c, world, u, rank) != ncclSuccess) return BCM3HIP_ERR_HIP;
    *comm = c;
    return 0;
}

int bcm3hip_nccl_comm_destroy(void* comm)
{
    return (!comm || ncclCommDestroy((ncclComm_t)comm) == ncclSuccess) ? 0 : BCM3HIP_ERR_HIP;
}

// one grouped round of point-to-point transfers: n_send sends (buffer, peer) and n_recv receives,
// count doubles each; posted in array order, so messages between one pair of ranks match in order
int bcm3hip_nccl_exchange(void* comm, int n_send, const double* const* send, const int* send_peer, int n_recv,
                          double* const* recv, const int* recv_peer, size_t count, void* stream)
{
    if (!comm || n_send < 0 || n_recv < 0) return BCM3HIP_ERR_ARG;
    if (ncclGroupStart() != ncclSuccess) return BCM3HIP_ERR_HIP;
    bool ok = true;
    for (int i = 0; i < n_send; i++)
        ok &= ncclSend(send[i], count, ncclDouble, send_peer[i], (ncclComm_t)comm, (hipStream_t)stream) == ncclSuccess;
    for (int i = 0; i < n_recv; i++)
        ok &= ncclRecv(recv[i], count, ncclDouble, recv_peer[i], (ncclComm_t)comm, (hipStream_t)stream) == ncclSuccess;
    ok &= ncclGroupEnd() == ncclSuccess;
    return ok ? 0 : BCM3HIP_ERR_HIP;
}

}  // extern "C"

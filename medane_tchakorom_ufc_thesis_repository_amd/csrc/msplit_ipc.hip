// msplit_ipc.hip -- HBM mailboxes shared between processes (HIP IPC over xGMI).
//
// The asynchronous transports (amsg.c, abcast.c) keep their control words in
// POSIX shared memory and, with device slots enabled, their payloads in the
// sender's HBM: the sender copies its plane / rows into its own slot, and a
// receiver on another GPU (or another process on the same GPU) copies them
// straight out of the sender's HBM over xGMI -- one device-to-device copy
// instead of HBM -> host -> HBM.  These helpers are the only HIP calls those
// C files make.
#include <hip/hip_runtime.h>

#include <cstring>

#include "msplit_ctx.hpp"

static_assert(sizeof(hipIpcMemHandle_t) <= MSPI_IPC_HANDLE_BYTES, "IPC handle size");

extern "C" int mspi_dev_alloc(msp_ctx* c, size_t bytes, void** p) {
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMalloc(p, bytes ? bytes : 8));
  HIPCHK(hipMemsetAsync(*p, 0, bytes ? bytes : 8, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_dev_free(void* p) {
  if (p) HIPCHK(hipFree(p));
  return MSP_SUCCESS;
}

extern "C" int mspi_ipc_export(void* p, uint8_t* handle) {
  hipIpcMemHandle_t h;
  HIPCHK(hipIpcGetMemHandle(&h, p));
  memset(handle, 0, MSPI_IPC_HANDLE_BYTES);
  memcpy(handle, &h, sizeof(h));
  return MSP_SUCCESS;
}

extern "C" int mspi_ipc_open(msp_ctx* c, const uint8_t* handle, void** p) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess));
  return MSP_SUCCESS;
}

extern "C" int mspi_ipc_close(void* p) {
  if (p) HIPCHK(hipIpcCloseMemHandle(p));
  return MSP_SUCCESS;
}

// device to device on the context's stream, no wait (either end may be a peer mapping)
extern "C" int mspi_d2d_async(msp_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!bytes) return MSP_SUCCESS;
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
  return MSP_SUCCESS;
}

// The address the GPU uses for a word of a registered host region (amsg.c's shared state words)
extern "C" int mspi_host_device_ptr(void* host, void** dev) {
  HIPCHK(hipHostGetDevicePointer(dev, host, 0));
  return MSP_SUCCESS;
}

extern "C" uint64_t mspi_stream_key(const msp_ctx* c) { return (uint64_t)(uintptr_t)c->stream; }

namespace {

// One lane stores v into a word of a registered host region, after everything before it on the stream: a
// system-scope release (the payload copies before it are complete and visible to other processes and GPUs
// when the word changes).  A vector store, one per launch.
template <typename T>
__global__ void k_publish(T* p, T v) {
  if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

extern "C" int mspi_stream_store_u64(msp_ctx* c, uint64_t* dev_word, uint64_t v) {
  k_publish<uint64_t><<<1, 64, 0, c->stream>>>(dev_word, v);
  HIPCHK(hipGetLastError());
  return MSP_SUCCESS;
}

extern "C" int mspi_stream_store_u32(msp_ctx* c, uint32_t* dev_word, uint32_t v) {
  k_publish<uint32_t><<<1, 64, 0, c->stream>>>(dev_word, v);
  HIPCHK(hipGetLastError());
  return MSP_SUCCESS;
}

// height rows of width bytes, pitched, device to device (either end may be a peer mapping), enqueued only
extern "C" int mspi_d2d_async2d(msp_ctx* c, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                                size_t height) {
  if (!width || !height) return MSP_SUCCESS;
  if (height == 1 || (dpitch == width && spitch == width))
    HIPCHK(hipMemcpyAsync(dst, src, width * height, hipMemcpyDeviceToDevice, c->stream));
  else
    HIPCHK(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice, c->stream));
  return MSP_SUCCESS;
}

// height rows of width bytes, pitched, device to device (either end may be a peer mapping)
extern "C" int mspi_d2d_sync(msp_ctx* c, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                             size_t height) {
  if (!width || !height) return MSP_SUCCESS;
  if (height == 1 || (dpitch == width && spitch == width))
    HIPCHK(hipMemcpyAsync(dst, src, width * height, hipMemcpyDeviceToDevice, c->stream));
  else
    HIPCHK(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MSP_SUCCESS;
}

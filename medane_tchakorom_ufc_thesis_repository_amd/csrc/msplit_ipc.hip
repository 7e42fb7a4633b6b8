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

// api_util.h — host helpers shared by the C-ABI sources (api.cpp, eval.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <new>
#include <string>

#include "shelfi_internal.h"

namespace shelfi {

// -------------------------------------------------------------- helpers ----
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev == dev) {  // the common case: nothing to switch (and nothing to restore)
      prev = -1;
      return;
    }
    SHELFI_HIP(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};


template <class F>
inline int guarded(F&& f) {
  try {
    f();
    return SHELFI_OK;
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("host out of memory");
    return SHELFI_ERR_DEVICE;
  } catch (const std::exception& e) {
    set_error(e.what());
    return SHELFI_ERR_DEVICE;
  }
}

inline void dfree(void*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
template <class T>
inline void dfree_t(T*& p) {
  void* v = p;
  dfree(v);
  p = nullptr;
}

inline void* ensure(void*& buf, size_t& cap, size_t bytes) {
  if (bytes <= cap && buf) return buf;
  dfree(buf);
  cap = 0;
  size_t want = bytes < 64 ? 64 : bytes;
  SHELFI_HIP(hipMalloc(&buf, want));
  cap = want;
  return buf;
}

template <class T>
inline T* upload(const T* host, size_t count) {
  void* d = nullptr;
  SHELFI_HIP(hipMalloc(&d, sizeof(T) * (count ? count : 1)));
  SHELFI_HIP(hipMemcpy(d, host, sizeof(T) * count, hipMemcpyHostToDevice));
  return (T*)d;
}

}  // namespace shelfi

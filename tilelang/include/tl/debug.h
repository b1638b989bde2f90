// tl/debug.h — device printing / assertions (reference src/tl_templates/hip/debug.h).
#pragma once

namespace tl {

TL_DEVICE void print_val(const char* msg, float v) {
  printf("%s: block(%d,%d,%d) thread(%d) = %f\n", msg, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z,
         (int)threadIdx.x, (double)v);
}
TL_DEVICE void print_val(const char* msg, double v) { print_val(msg, (float)v); }
TL_DEVICE void print_val(const char* msg, half_t v) { print_val(msg, (float)v); }
TL_DEVICE void print_val(const char* msg, bfloat16_t v) { print_val(msg, (float)v); }
TL_DEVICE void print_val(const char* msg, int v) {
  printf("%s: block(%d,%d,%d) thread(%d) = %d\n", msg, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z,
         (int)threadIdx.x, v);
}
TL_DEVICE void print_val(const char* msg, long v) { print_val(msg, (int)v); }
TL_DEVICE void print_val(const char* msg, unsigned v) { print_val(msg, (int)v); }
TL_DEVICE void print_val(const char* msg, bool v) { print_val(msg, (int)v); }

template <typename T> TL_DEVICE void print_buffer(const char* msg, const char* name, const T* buf, int n) {
  for (int i = 0; i < n; ++i)
    printf("%s %s[%d] block(%d,%d,%d) thread(%d) = %f\n", msg, name, i, (int)blockIdx.x, (int)blockIdx.y,
           (int)blockIdx.z, (int)threadIdx.x, (double)(float)buf[i]);
}

TL_DEVICE void device_assert(bool cond, const char* msg) {
  if (!cond) {
    printf("tilelang device assert failed: %s (block %d,%d,%d thread %d)\n", msg, (int)blockIdx.x, (int)blockIdx.y,
           (int)blockIdx.z, (int)threadIdx.x);
    __builtin_trap();
  }
}

}  // namespace tl

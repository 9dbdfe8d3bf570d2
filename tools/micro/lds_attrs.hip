// Prints the device's LDS limits as HIP reports them (which attribute bqg_create can size
// check_launch from).
#include <hip/hip_runtime.h>
#include <cstdio>

int main() {
  int v = 0;
  const struct { hipDeviceAttribute_t a; const char* n; } attrs[] = {
      {hipDeviceAttributeMaxSharedMemoryPerBlock, "MaxSharedMemoryPerBlock"},
      {hipDeviceAttributeSharedMemPerBlockOptin, "SharedMemPerBlockOptin"},
      {hipDeviceAttributeSharedMemPerMultiprocessor, "SharedMemPerMultiprocessor"},
      {hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, "MaxSharedMemoryPerMultiprocessor"},
  };
  for (const auto& x : attrs) {
    v = -1;
    const hipError_t e = hipDeviceGetAttribute(&v, x.a, 0);
    printf("%-34s %d (%s)\n", x.n, v, hipGetErrorString(e));
  }
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess)
    printf("prop sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu gcnArchName %s\n", p.sharedMemPerBlock,
           p.maxSharedMemoryPerMultiProcessor, p.gcnArchName);
  return 0;
}

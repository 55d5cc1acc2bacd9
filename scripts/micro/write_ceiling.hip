// Write-stream ceiling on MI355X for the assembly's output size (CSR values + rhs + dq,
// ~43.6 MB at C3): plain / 16-byte / nontemporal stores, several grid shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -o write_ceiling write_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
// WRITE_SIZE calibration (scripts/gpu_run.sh wcal): every kernel writes exactly `bytes`, 55
// launches each; rocprofv3 --pmc WRITE_SIZE per kernel / bytes = the counter's factor.

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__global__ void w1(double* p, long n, double v) {  // one double per thread
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}
__global__ void w1sc1(double* p, long n, double v) {  // one double per thread, write-through
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p + i),
                       __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void w2(double2* p, long n2, double v) {  // 16 B per thread
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n2) p[i] = make_double2(v, v);
}
__global__ void w2nt(double2* p, long n2, double v) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n2) { __builtin_nontemporal_store(v, &p[i].x); __builtin_nontemporal_store(v, &p[i].y); }
}
template <int K>
__global__ void wk(double* p, long n, double v) {  // K doubles per thread, wave-strided
  long base = ((long)blockIdx.x * blockDim.x) * K + threadIdx.x;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    long i = base + (long)k * blockDim.x;
    if (i < n) p[i] = v;
  }
}
__global__ void wgrid(double* p, long n, double v) {  // grid-stride, fixed grid
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}

int main(int argc, char** argv) {
  long bytes = argc > 1 ? atol(argv[1]) : 43645616;
  long n = bytes / 8;
  int reps = 50;
  double* p;
  CK(hipMalloc(&p, n * 8 + 4096));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 5; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e9, tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(a)); launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best; tot += ms;
    }
    printf("%-28s avg %7.2f us  best %7.2f us  %6.0f GB/s (avg)\n", name, tot / reps * 1e3, best * 1e3,
           bytes / (tot / reps * 1e-3) / 1e9);
  };
  run("w1 256", [&] { w1<<<(n + 255) / 256, 256>>>(p, n, 1.0); });
  run("w1 1024", [&] { w1<<<(n + 1023) / 1024, 1024>>>(p, n, 1.0); });
  run("w1sc1 1024", [&] { w1sc1<<<(n + 1023) / 1024, 1024>>>(p, n, 1.0); });
  run("w2 256", [&] { w2<<<(n / 2 + 255) / 256, 256>>>((double2*)p, n / 2, 1.0); });
  run("w2nt 256", [&] { w2nt<<<(n / 2 + 255) / 256, 256>>>((double2*)p, n / 2, 1.0); });
  run("wk<4> 256", [&] { wk<4><<<(n + 1023) / 1024, 256>>>(p, n, 1.0); });
  run("wk<8> 256", [&] { wk<8><<<(n + 2047) / 2048, 256>>>(p, n, 1.0); });
  run("wk<16> 256", [&] { wk<16><<<(n + 4095) / 4096, 256>>>(p, n, 1.0); });
  for (int g : {1024, 2048, 4096, 8192})
  { char nm[64]; snprintf(nm, 64, "wgrid %d x 256", g); run(nm, [&] { wgrid<<<g, 256>>>(p, n, 1.0); }); }
  run("hipMemsetAsync", [&] { CK(hipMemsetAsync(p, 0, n * 8)); });
  // launch overhead floor
  run("empty w1 (n=1)", [&] { w1<<<1, 64>>>(p, 1, 1.0); });
  return 0;
}

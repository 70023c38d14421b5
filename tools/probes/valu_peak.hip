// Vector-ALU peak probe: what FLOP/clk/SIMD do fp64 FMA, fp32 FMA, packed
// fp32 FMA and packed fp16 FMA reach on gfx950?  The precision counter pass
// divides SQ_INSTS_VALU_FLOPS_FPxx by SIMD-cycles x a per-precision peak
// (SlotDerive.h, makeAgentConsts); this pins those peaks by measurement.
//
// Each lane runs 8 independent FMA chains (enough ILP to hide the VALU
// dependency latency with 8 waves per SIMD); the store guard compares with a
// run-time value so no chain is dead.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/probes/valu_peak.hip -o build/probes/valu_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <typename T>
__device__ __forceinline__ T fma_(T a, T b, T c) {
  return a * b + c;
}

template <typename T>
__global__ __launch_bounds__(256) void burn(T* out, int iters, T b, T c, float sentinel) {
  T x0 = b * (T)(threadIdx.x), x1 = x0 + c, x2 = x1 + c, x3 = x2 + c;
  T x4 = x3 + c, x5 = x4 + c, x6 = x5 + c, x7 = x6 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x0 = fma_(x0, b, c);
      x1 = fma_(x1, b, c);
      x2 = fma_(x2, b, c);
      x3 = fma_(x3, b, c);
      x4 = fma_(x4, b, c);
      x5 = fma_(x5, b, c);
      x6 = fma_(x6, b, c);
      x7 = fma_(x7, b, c);
    }
  }
  T s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (static_cast<float>(s[0]) == sentinel) out[threadIdx.x] = s;
}

// scalar (non-vector) variants: fp32 and fp64 FMA
template <typename T>
__global__ __launch_bounds__(256) void burn1(T* out, int iters, T b, T c, float sentinel) {
  T x0 = b * (T)(threadIdx.x), x1 = x0 + c, x2 = x1 + c, x3 = x2 + c;
  T x4 = x3 + c, x5 = x4 + c, x6 = x5 + c, x7 = x6 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x0 = fma_(x0, b, c);
      x1 = fma_(x1, b, c);
      x2 = fma_(x2, b, c);
      x3 = fma_(x3, b, c);
      x4 = fma_(x4, b, c);
      x5 = fma_(x5, b, c);
      x6 = fma_(x6, b, c);
      x7 = fma_(x7, b, c);
    }
  }
  T s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (static_cast<float>(s) == sentinel) out[threadIdx.x] = s;
}

template <typename K>
double timeIt(K launch) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 5.0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount, simds = cus * 4;
  const double ghz = p.clockRate * 1e-6;  // kHz -> GHz (the max engine clock)
  printf("%s: %d CUs, %d SIMDs, max sclk %.3f GHz\n", p.gcnArchName, cus, simds, ghz);
  void* out;
  CHECK(hipMalloc(&out, 1 << 16));
  const int blocks = cus * 8, iters = 20000;  // 8 waves x ... per CU: 2 waves / SIMD per block wave
  const double lanes = static_cast<double>(blocks) * 256;
  const double fmaPerLane = static_cast<double>(iters) * 4 * 8;
  struct Row {
    const char* name;
    double flopsPerFma;  // per lane FMA instruction
    double ms;
  } rows[4];
  rows[0] = {"fp64 fma", 2, timeIt([&] {
               hipLaunchKernelGGL(burn1<double>, dim3(blocks), dim3(256), 0, 0, (double*)out, iters, 0.9999, 1e-6, -1.f);
             })};
  rows[1] = {"fp32 fma", 2, timeIt([&] {
               hipLaunchKernelGGL(burn1<float>, dim3(blocks), dim3(256), 0, 0, (float*)out, iters, 0.9999f, 1e-6f, -1.f);
             })};
  f32x2 b2 = {0.9999f, 0.9998f}, c2 = {1e-6f, 2e-6f};
  rows[2] = {"fp32 packed (v_pk_fma_f32)", 4, timeIt([&] {
               hipLaunchKernelGGL(burn<f32x2>, dim3(blocks), dim3(256), 0, 0, (f32x2*)out, iters, b2, c2, -1.f);
             })};
  f16x2 h2 = {(_Float16)0.999f, (_Float16)0.998f}, hc = {(_Float16)1e-3f, (_Float16)2e-3f};
  rows[3] = {"fp16 packed (v_pk_fma_f16)", 4, timeIt([&] {
               hipLaunchKernelGGL(burn<f16x2>, dim3(blocks), dim3(256), 0, 0, (f16x2*)out, iters, h2, hc, -1.f);
             })};
  for (const auto& r : rows) {
    const double flops = lanes * fmaPerLane * r.flopsPerFma;
    const double tf = flops / (r.ms * 1e-3) * 1e-12;
    printf("%-28s %8.3f ms  %7.1f TFLOP/s  %6.1f FLOP/clk/SIMD at max sclk\n", r.name, r.ms, tf,
           flops / (r.ms * 1e-3) / (simds * ghz * 1e9));
  }
  CHECK(hipFree(out));
  return 0;
}

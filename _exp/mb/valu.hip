// micro-benchmark: wave64 VALU issue rate for f32 ops on gfx950 (diagnostic, not product)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int OP>
__global__ __launch_bounds__(256) void k(float* out, float a, int iters) {
    float x[8];
    f2 y[8];
    for (int i = 0; i < 8; ++i) { x[i] = a + threadIdx.x + i; y[i] = f2{x[i], x[i] + 1.f}; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 7]));
            if (OP == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(y[i]) : "v"(y[(i + 1) & 7]));
            if (OP == 2) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(x[(i + 1) & 7]), "v"(x[(i + 2) & 7]));
            if (OP == 3) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[i]) : "v"(x[(i + 1) & 7]));
        }
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i] + y[i].x + y[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    float* out;
    hipMalloc(&out, 4 << 20);
    const int blocks = 256 * 8, iters = 4096;
    const char* names[4] = {"v_sub_f32", "v_pk_add_f32", "v_max3_f32", "v_max_f32"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep)
        for (int op = 0; op < 4; ++op) {
            hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 1.f, iters);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 1.f, iters);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 1.f, iters);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 1.f, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double winstr = (double)blocks * 4 * iters * 8;  // wave-instructions
            double simd_cycles = 1024.0 * 2.4e6 * ms;        // 1024 SIMDs at 2.4 GHz (nominal)
            if (rep) printf("%-14s %.3f ms  cycles per wave64 instr per SIMD: %.2f\n", names[op], ms, simd_cycles / winstr);
        }
    return 0;
}

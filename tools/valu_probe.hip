// valu_probe: issue rate of the VALU operations the normalising histogram build is made of
// (development tool, round 6).  Each kernel runs 8 independent chains per lane of one operation
// for ITER iterations; 4 waves per SIMD on every CU.  Reported: wave-instructions per cycle per
// SIMD (1.0 = one per clock) from the kernel time and the GPU clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITER 4096
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void __launch_bounds__(256) k_op(uint32_t *out, uint32_t seed) {
	uint32_t u[8];
	double d[8];
	f32x2 f[8];
	for (int i = 0; i < 8; i++) {
		u[i] = seed ^ (threadIdx.x * 8 + i);
		d[i] = (double)u[i];
		f[i] = f32x2{(float)u[i], (float)(u[i] + 1)};
	}
	const double a = 1.0000123 + seed * 1e-12, b = 0.4999;
	const f32x2 fa = {1.0001f, 0.9999f}, fb = {0.25f, 0.75f};
	for (int it = 0; it < ITER; it++) {
#pragma unroll
		for (int i = 0; i < 8; i++) {
			/* asm volatile: the operation is issued as written, 8 independent chains per lane */
			if (OP == 0)
				asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(u[i]));
			else if (OP == 1)
				asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(u[i]) : "v"(d[i]));
			else if (OP == 2)
				asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(a));
			else if (OP == 3)
				asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(b));
			else if (OP == 4)
				asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fa), "v"(fb));
			else if (OP == 5)
				asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(it));
			else if (OP == 6)
				asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(it), "v"(0x05040100u));
			else if (OP == 7)
				asm volatile("v_floor_f32 %0, %0" : "+v"(f[i].x));
		}
	}
	uint32_t r = 0;
	for (int i = 0; i < 8; i++)
		r ^= u[i] ^ (uint32_t)d[i] ^ __builtin_bit_cast(uint32_t, f[i].x) ^ __builtin_bit_cast(uint32_t, f[i].y);
	if (r == 0x12345678u)
		out[0] = r;
}

template <int OP>
static void run(const char *name, uint32_t *o, int cus, double ghz) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const int grid = cus * 4;	/* 4 workgroups of 4 waves per CU: 4 waves per SIMD */
	hipLaunchKernelGGL(k_op<OP>, dim3(grid), dim3(256), 0, 0, o, 1u);
	(void)hipDeviceSynchronize();
	(void)hipEventRecord(a);
	for (int r = 0; r < 5; r++)
		hipLaunchKernelGGL(k_op<OP>, dim3(grid), dim3(256), 0, 0, o, (uint32_t)r + 2u);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 5;
	/* wave-instructions per SIMD: 4 waves x ITER x 8 */
	const double winstr = 4.0 * ITER * 8;
	const double cycles = ms * 1e-3 * ghz * 1e9;
	printf("%-16s %8.3f ms  %.3f wave-instructions / cycle / SIMD (%s)\n", name, ms, winstr / cycles,
			hipGetErrorString(hipGetLastError()));
}

int main() {
	uint32_t *o;
	(void)hipMalloc(&o, 64);
	hipDeviceProp_t pr;
	(void)hipGetDeviceProperties(&pr, 0);
	const double ghz = pr.clockRate / 1e6;
	printf("%s: %d CUs, clock %.2f GHz\n", pr.gcnArchName, pr.multiProcessorCount, ghz);
	for (int rep = 0; rep < 2; rep++) {
		run<0>("v_cvt_f64_u32", o, pr.multiProcessorCount, ghz);
		run<1>("v_cvt_u32_f64", o, pr.multiProcessorCount, ghz);
		run<2>("v_mul_f64", o, pr.multiProcessorCount, ghz);
		run<3>("v_add_f64", o, pr.multiProcessorCount, ghz);
		run<4>("v_pk_fma_f32", o, pr.multiProcessorCount, ghz);
		run<5>("v_add_u32", o, pr.multiProcessorCount, ghz);
		run<6>("v_perm_b32", o, pr.multiProcessorCount, ghz);
		run<7>("v_floor_f32", o, pr.multiProcessorCount, ghz);
	}
	return 0;
}

// bw_probe2: which structural feature of k_stack_hist costs bandwidth (development tool).
// Pattern: 262144 workgroups of 256 threads, each reads a 128-byte row segment of a
// 4096x4096 u16 plane from all 512 frames (16 GiB), 4 waves x 128 frames.
//   LDS   : dynamic LDS bytes allocated per workgroup (limits occupancy)
//   BUF   : 1 = per-frame buffer descriptors + raw_buffer_load_b16, 0 = global loads
//   PRO   : 1 = every wave first loads frames 0..15 and waits for them + a barrier
//   BATCH : loads per batch (double-buffered when DB = 1)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define NF 512
#define ROWB 8192
#define NROW 4096
#define FRAMEB ((size_t)ROWB * NROW)

template <int BUF, int PRO, int BATCH, int DB>
__global__ void __launch_bounds__(256) k_probe(const char *__restrict__ base, unsigned *__restrict__ out) {
	extern __shared__ unsigned lds[];
	const int seg = blockIdx.x & 63, row = blockIdx.x >> 6;
	const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const size_t off = (size_t)row * ROWB + (size_t)seg * 128 + lane * 2;
	unsigned acc = 0;
	auto ld = [&](int f) -> unsigned {
		if (BUF) {
			const char *fb = base + (size_t)f * FRAMEB;
			auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)fb, (short)0, (int)FRAMEB, 0x00020000);
			return (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rs, (int)(row * ROWB + seg * 128 + lane * 2), 0, 0);
		}
		return *(const unsigned short *)(base + (size_t)f * FRAMEB + off);
	};
	if (PRO) {
		unsigned v[16];
#pragma unroll
		for (int k = 0; k < 16; k++) v[k] = ld(k);
#pragma unroll
		for (int k = 0; k < 16; k++) acc += v[k];
		lds[threadIdx.x] = acc;
		__syncthreads();
		acc += lds[(threadIdx.x + 64) & 255];
	}
	unsigned a[BATCH], b[BATCH];
	int f0 = wave * BATCH;
	const int step = 4 * BATCH;
#pragma unroll
	for (int u = 0; u < BATCH; u++) a[u] = ld(f0 + u);
	for (; f0 < NF; f0 += 2 * step) {
		const int n1 = f0 + step < NF ? f0 + step : f0;
#pragma unroll
		for (int u = 0; u < BATCH; u++) b[u] = ld(n1 + u);
#pragma unroll
		for (int u = 0; u < BATCH; u++) acc += a[u];
		if (f0 + step >= NF) break;
		const int n2 = f0 + 2 * step < NF ? f0 + 2 * step : f0 + step;
#pragma unroll
		for (int u = 0; u < BATCH; u++) a[u] = ld(n2 + u);
#pragma unroll
		for (int u = 0; u < BATCH; u++) acc += b[u];
	}
	if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(unsigned *p, size_t n) {
	for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		p[i] = (unsigned)(i * 2654435761u);
}

template <int BUF, int PRO, int BATCH, int DB>
static void run(const char *d, unsigned *o, int lds, const char *name) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const int grid = NROW * 64;
	(void)hipFuncSetAttribute((const void *)k_probe<BUF, PRO, BATCH, DB>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
	hipLaunchKernelGGL((k_probe<BUF, PRO, BATCH, DB>), dim3(grid), dim3(256), lds, 0, d, o);
	(void)hipDeviceSynchronize();
	(void)hipEventRecord(a);
	for (int i = 0; i < 3; i++)
		hipLaunchKernelGGL((k_probe<BUF, PRO, BATCH, DB>), dim3(grid), dim3(256), lds, 0, d, o);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 3;
	printf("%-34s lds=%6d: %7.3f ms %7.1f GB/s  (%s)\n", name, lds, ms, (double)NF * FRAMEB / ms / 1e6,
			hipGetErrorString(hipGetLastError()));
}

int main() {
	char *d;
	unsigned *o;
	if (hipMalloc(&d, (size_t)NF * FRAMEB) != hipSuccess) {
		printf("alloc failed\n");
		return 1;
	}
	(void)hipMalloc(&o, 64);
	hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (unsigned *)d, (size_t)NF * FRAMEB / 4);
	(void)hipDeviceSynchronize();
	run<0, 0, 8, 1>(d, o, 1024, "global b8");
	run<0, 0, 16, 1>(d, o, 1024, "global b16");
	run<1, 0, 16, 1>(d, o, 1024, "buffer b16");
	run<1, 0, 16, 1>(d, o, 23552, "buffer b16 occ6");
	run<1, 1, 16, 1>(d, o, 1024, "buffer b16 prologue");
	run<1, 1, 16, 1>(d, o, 23552, "buffer b16 prologue occ6");
	run<0, 1, 16, 1>(d, o, 23552, "global b16 prologue occ6");
	run<1, 0, 8, 1>(d, o, 23552, "buffer b8 occ6");
	run<1, 0, 32, 1>(d, o, 23552, "buffer b32 occ6");
	return 0;
}

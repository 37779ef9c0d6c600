// bw_probe3: cost of shifted (non 128-B aligned) row loads vs load width (development tool).
// 512 frames of 4096x4096 u16; each workgroup (4 waves) reads one TB-byte row segment of
// every frame (frames split over the waves, 16-load double-buffered batches) at a per-frame
// byte shift: SH = 0 none, 1 = even pixel shifts (4-B aligned), 2 = any pixel shift.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define NF 512
#define ROWB 8192
#define NROW 4096
#define FRAMEB ((size_t)ROWB * NROW)

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int shift_of(int f, int SH) {
	if (SH == 0)
		return 0;
	int s = (int)((f * 2654435761u) >> 27) - 16;	/* -16..15 pixels */
	if (SH == 1)
		s &= ~1;
	return 2 * s;
}

template <int W, int SH>	/* W = dwords per lane: 1, 2, 4 */
__global__ void __launch_bounds__(256) k_probe(const char *__restrict__ base, unsigned *__restrict__ out) {
	constexpr int TB = 256 * W;
	constexpr int NSEG = ROWB / TB;
	const int seg = blockIdx.x % NSEG, row = blockIdx.x / NSEG;
	const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int edge = (seg == 0 || seg == NSEG - 1);
	unsigned acc = 0;
	auto ld = [&](int f) -> unsigned {
		const char *fb = base + (size_t)f * FRAMEB;
		auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)fb, (short)0, (int)FRAMEB, 0x00020000);
		const int o = row * ROWB + seg * TB + lane * 4 * W - (edge ? 0 : shift_of(f, SH));
		if (W == 1)
			return __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
		if (W == 2) {
			u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 0);
			return v.x ^ v.y;
		}
		u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
		return v.x ^ v.y ^ v.z ^ v.w;
	};
	constexpr int BATCH = 16;
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

template <int W, int SH>
static void run(const char *d, unsigned *o) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const int grid = NROW * (ROWB / (256 * W));
	hipLaunchKernelGGL((k_probe<W, SH>), dim3(grid), dim3(256), 0, 0, d, o);
	(void)hipDeviceSynchronize();
	(void)hipEventRecord(a);
	for (int i = 0; i < 3; i++)
		hipLaunchKernelGGL((k_probe<W, SH>), dim3(grid), dim3(256), 0, 0, d, o);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 3;
	printf("dwords/lane=%d shift=%d: %7.3f ms %7.1f GB/s  (%s)\n", W, SH, ms, (double)NF * FRAMEB / ms / 1e6,
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
	run<1, 0>(d, o);
	run<1, 1>(d, o);
	run<1, 2>(d, o);
	run<2, 0>(d, o);
	run<2, 1>(d, o);
	run<2, 2>(d, o);
	run<4, 0>(d, o);
	run<4, 1>(d, o);
	run<4, 2>(d, o);
	return 0;
}

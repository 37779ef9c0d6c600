// bw_probe: HBM read bandwidth of the stacking access pattern on gfx950 (development tool).
// A 16 GiB "sequence" of 512 frames (32 MiB each, one 4096x4096 u16 plane) is read in the
// order a pixel-tile kernel reads it: each workgroup owns a segment of SEG bytes of one
// row and reads that segment from all 512 frames.  Variants: load width per lane and SEG.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define NF 512
#define ROWB 8192              /* bytes per row: 4096 u16 */
#define NROW 4096
#define FRAMEB ((size_t)ROWB * NROW)

template <int SEGB, int LW>   /* segment bytes per frame row, load width per lane (bytes) */
__global__ void __launch_bounds__(256) k_probe(const char *__restrict__ base, unsigned *__restrict__ out) {
	constexpr int LANES_PER_SEG = SEGB / LW;          /* lanes covering one frame segment */
	constexpr int FR_PER_WAVE = 64 / LANES_PER_SEG;   /* frames per wave instruction */
	const int nseg = ROWB / SEGB;
	const int seg = blockIdx.x % nseg, row = blockIdx.x / nseg;
	const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	const int fsub = lane / LANES_PER_SEG, part = lane % LANES_PER_SEG;
	unsigned acc = 0;
	const char *p0 = base + (size_t)row * ROWB + (size_t)seg * SEGB + part * LW;
	for (int f0 = wave * FR_PER_WAVE; f0 < NF; f0 += 4 * FR_PER_WAVE * 8) {
		unsigned v[8];
#pragma unroll
		for (int u = 0; u < 8; u++) {
			const int f = f0 + u * 4 * FR_PER_WAVE + fsub;
			const char *p = p0 + (size_t)(f < NF ? f : NF - 1) * FRAMEB;
			if (LW == 2) v[u] = *(const unsigned short *)p;
			else if (LW == 4) v[u] = *(const unsigned *)p;
			else if (LW == 8) { uint2 t = *(const uint2 *)p; v[u] = t.x ^ t.y; }
			else { uint4 t = *(const uint4 *)p; v[u] = t.x ^ t.y ^ t.z ^ t.w; }
		}
#pragma unroll
		for (int u = 0; u < 8; u++) acc += v[u];
	}
	if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(unsigned *p, size_t n) {
	for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		p[i] = (unsigned)(i * 2654435761u);
}

template <int SEGB, int LW>
static void run(const char *d, unsigned *o, const char *name) {
	hipEvent_t a, b;
	hipEventCreate(&a); hipEventCreate(&b);
	const int grid = NROW * (ROWB / SEGB);
	hipLaunchKernelGGL((k_probe<SEGB, LW>), dim3(grid), dim3(256), 0, 0, d, o);
	hipDeviceSynchronize();
	hipEventRecord(a);
	for (int i = 0; i < 3; i++)
		hipLaunchKernelGGL((k_probe<SEGB, LW>), dim3(grid), dim3(256), 0, 0, d, o);
	hipEventRecord(b);
	hipEventSynchronize(b);
	float ms; hipEventElapsedTime(&ms, a, b); ms /= 3;
	printf("%-28s seg=%5d B lw=%2d: %8.3f ms  %7.1f GB/s\n", name, SEGB, LW, ms, (double)NF * FRAMEB / ms / 1e6);
}

int main() {
	char *d; unsigned *o;
	if (hipMalloc(&d, (size_t)NF * FRAMEB) != hipSuccess) { printf("alloc failed\n"); return 1; }
	hipMalloc(&o, 64);
	hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (unsigned *)d, (size_t)NF * FRAMEB / 4);
	hipDeviceSynchronize();
	run<128, 2>(d, o, "tile64 u16 (current)");
	run<128, 4>(d, o, "tile64 dword");
	run<128, 16>(d, o, "tile64 dwordx4");
	run<256, 4>(d, o, "tile128 dword");
	run<512, 8>(d, o, "tile256 dwordx2");
	run<512, 16>(d, o, "tile256 dwordx4");
	run<1024, 16>(d, o, "tile512 dwordx4");
	run<2048, 16>(d, o, "tile1024 dwordx4");
	run<8192, 16>(d, o, "row dwordx4");
	hipFree(d);
	return 0;
}

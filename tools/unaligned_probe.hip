// unaligned_probe: do 4-byte buffer / global loads at 2-byte aligned addresses return the
// bytes at that address on gfx950 (needed for 2-pixels-per-lane loads of shifted frames)?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(const uint16_t *src, uint32_t *out_buf, uint32_t *out_glb) {
	const int l = threadIdx.x;
	const uint32_t off = 2u * (uint32_t)l + 2u;	/* odd element index: 2-byte aligned */
	auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, 4096, 0x00020000);
	out_buf[l] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0);
	uint32_t v;
	__builtin_memcpy(&v, (const char *)src + off, 4);
	out_glb[l] = v;
}

int main() {
	uint16_t h[2048];
	for (int i = 0; i < 2048; i++) h[i] = (uint16_t)(i * 3 + 1);
	uint16_t *d; uint32_t *ob, *og;
	(void)hipMalloc(&d, sizeof h); (void)hipMalloc(&ob, 256); (void)hipMalloc(&og, 256);
	(void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
	hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, ob, og);
	uint32_t rb[64], rg[64];
	(void)hipMemcpy(rb, ob, 256, hipMemcpyDeviceToHost);
	(void)hipMemcpy(rg, og, 256, hipMemcpyDeviceToHost);
	int okb = 0, okg = 0;
	for (int l = 0; l < 64; l++) {
		const uint32_t want = (uint32_t)h[l + 1] | ((uint32_t)h[l + 2] << 16);
		okb += rb[l] == want;
		okg += rg[l] == want;
	}
	printf("buffer dword at 2-byte offsets: %d/64 correct (lane0 got %08x want %08x)\n", okb, rb[0],
			(uint32_t)h[1] | ((uint32_t)h[2] << 16));
	printf("global dword at 2-byte offsets: %d/64 correct\n", okg);
	return 0;
}

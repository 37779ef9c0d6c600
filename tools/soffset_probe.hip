// soffset_probe: is the SGPR offset of a raw buffer load part of the bounds check on gfx950?
// A 1 KiB buffer of 0xABABABAB, a descriptor with num_records = 64 bytes; lanes load dword
// voffset = 4 lane with soffset 0 and soffset 128.  If soffset is range-checked, every lane
// of the soffset-128 load reads 0; otherwise lanes 0..15 (voffset < 64) read 0xABABABAB.
// Then soffset = 2^32 - 64 with voffset = 4 lane + 64: if voffset + soffset wraps in 32 bits
// (address and bounds check alike), lanes 0..15 read data again.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_probe(const unsigned *buf, unsigned *out, int soff, int vbias) {
	auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)0, 64, 0x00020000);
	const int lane = threadIdx.x;
	out[lane] = __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4 + vbias, soff, 0);
}

int main() {
	unsigned *b, *o, h[64];
	if (hipMalloc(&b, 1024) != hipSuccess || hipMalloc(&o, 256) != hipSuccess)
		return 1;
	(void)hipMemset(b, 0xAB, 1024);
	const int soffs[3] = {0, 128, -64}, vb[3] = {0, 0, 64};
	for (int t = 0; t < 3; t++) {
		const int soff = soffs[t];
		(void)hipMemset(o, 0x11, 256);
		hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, b, o, soff, vb[t]);
		if (hipMemcpy(h, o, 256, hipMemcpyDeviceToHost) != hipSuccess)
			return 2;
		int nz = 0, first0 = -1;
		for (int i = 0; i < 64; i++) {
			nz += h[i] != 0;
			if (h[i] == 0 && first0 < 0)
				first0 = i;
		}
		printf("soffset %3d voffset bias %2d: %d lanes read data (first zero lane %d), lane0 %08x lane15 %08x lane16 %08x\n", soff, vb[t], nz, first0, h[0], h[15], h[16]);
	}
	return 0;
}

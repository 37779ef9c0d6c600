// bw_probe4: load floor of the histogram stacking kernel's access pattern (development tool).
// 512 frames of 4096x4096 u16 (16 GiB) with per-frame registration shifts (the bench's
// synthetic shifts, |sx|, |sy| <= 16): a tile is a TW-byte segment of one output row; every
// frame contributes the row segment shifted by (sx, sy) (buffer loads, out-of-frame rows read
// 0 from the bounds check).  Tiles are dealt XCD-major as in k_stack_hist.  Variants: tile
// width and load width, waves per workgroup, register buffers of 16 frames per wave, LDS per
// workgroup (occupancy), and persistent workgroups that stream their tiles back to back.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NF 512
#define W 4096
#define H 4096
#define FRAMEB ((size_t)W * H * 2)

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Shift {
	int c1;	/* -(sy * W * 2 + 2 * sx) */
};

static uint64_t mix64(uint64_t z) {
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

template <int LW>
__device__ __forceinline__ unsigned ld1(const char *fb, int off) {
	auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)fb, (short)0, (int)FRAMEB, 0x00020000);
	if (LW == 4)
		return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
	if (LW == 8) {
		u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
		return v.x ^ v.y;
	}
	u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
	return v.x ^ v.y ^ v.z ^ v.w;
}

/* TW bytes per tile row, LW bytes per lane and instruction (TW / (64 LW) instructions per
 * frame), NBUF buffers of 16 frames, PERSIST: workgroups loop over their tiles */
template <int TW, int LW, int NBUF, bool PERSIST, int M>
__global__ void __launch_bounds__(1024) k_probe(const char *__restrict__ base, const int *__restrict__ c1,
		unsigned *__restrict__ out, int ntiles_total) {
	extern __shared__ unsigned lds[];
	constexpr int NI = TW / (64 * LW);	/* load instructions per frame */
	const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int nw = blockDim.x >> 6;
	const int ntx = (W * 2) / TW;
	const int nblk = (int)gridDim.x, xcd = (int)blockIdx.x & 7;
	/* tiles of this XCD: a contiguous range, dealt over its workgroups */
	const int per_xcd = ntiles_total / 8;
	const int t_lo = xcd * per_xcd, t_hi = t_lo + per_xcd;
	const int wg_in_xcd = (int)blockIdx.x >> 3, nwg_xcd = nblk >> 3;
	unsigned acc = 0;
	int tile = t_lo + wg_in_xcd;
	const int bpw = (NF / M - wave + nw - 1) / nw;	/* blocks of this wave per tile (blocks dealt round-robin) */
	/* flattened stream of (tile, block) items of this wave */
	auto item_off = [&](int t, int k, int m) -> int {
		const int xt = t % ntx, R = t / ntx;
		const int f = (wave + k * nw) * M + m;
		return R * W * 2 + xt * TW + lane * LW + c1[f];
	};
	auto frame_of = [&](int k, int m) { return (wave + k * nw) * M + m; };
	unsigned buf[NBUF][M * NI];
	int bt[NBUF], bk[NBUF];
	int t = tile, k = 0;
	auto next = [&]() {
		if (++k == bpw) {
			k = 0;
			t = PERSIST ? t + nwg_xcd : t_hi;
		}
	};
	auto load = [&](int s) {
		bt[s] = t;
		bk[s] = k;
		if (t < t_hi) {
#pragma unroll
			for (int m = 0; m < M; m++) {
				const char *fb = base + (size_t)frame_of(k, m) * FRAMEB;
				const int o = item_off(t, k, m);
#pragma unroll
				for (int i = 0; i < NI; i++)
					buf[s][m * NI + i] = ld1<LW>(fb, o + i * 64 * LW);
			}
		}
		next();
	};
#pragma unroll
	for (int s = 0; s < NBUF; s++)
		load(s);
	for (;;) {
		bool any = false;
#pragma unroll
		for (int s = 0; s < NBUF; s++) {
			if (bt[s] >= t_hi)
				continue;
			any = true;
#pragma unroll
			for (int j = 0; j < M * NI; j++)
				acc ^= buf[s][j];
			load(s);
		}
		if (!any)
			break;
	}
	if (acc == 0x12345678u)
		out[0] = acc + lds[0];
}

/* mode 6 (round 6): the same 256-B shifted row segments staged by LDS-DMA
 * (buffer_load_dword ... lds: per-lane source address, the wave's 64 dwords land lane-linear in
 * LDS) into a per-wave ring of NSLOT slots of 8 frames; the consumer reads each frame's dword back
 * with ds_read_b32 (what the binning would read instead of the load's VGPR).  The wait before a
 * slot's reads is a counted vmcnt leaving the younger slots' DMAs in flight.  LDSX = LDS bytes per
 * workgroup besides the ring (the histogram's 34.5 KB, or less to probe occupancy). */
typedef __attribute__((address_space(3))) void lds_void;

template <int NSLOT>
__global__ void __launch_bounds__(256) k_probe_lds(const char *__restrict__ base, const int *__restrict__ c1,
		unsigned *__restrict__ out, int ntiles_total, int check_tile) {
	extern __shared__ unsigned lds[];
	constexpr int M = 8, TW = 256;
	const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int nw = 4;
	const int ntx = (W * 2) / TW;
	const int xcd = (int)blockIdx.x & 7;
	const int per_xcd = ntiles_total / 8;
	const int t = xcd * per_xcd + ((int)blockIdx.x >> 3);
	const int xt = t % ntx, R = t / ntx;
	unsigned *ring = lds + wave * (NSLOT * M * 64);	/* this wave's slots: [slot][frame][lane] dwords */
	const int nblk = NF / M / nw;			/* blocks of 8 frames per wave */
	unsigned acc = 0;
	auto issue = [&](int k) {
		const int s = k % NSLOT;
#pragma unroll
		for (int m = 0; m < M; m++) {
			const int f = (wave + k * nw) * M + m;
			auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(base + (size_t)f * FRAMEB), (short)0, (int)FRAMEB,
					0x00020000);
			const int so = R * W * 2 + xt * TW + c1[f];
			__builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(ring + (s * M + m) * 64), 4, lane * 4, so, 0, 0);
		}
	};
#pragma unroll
	for (int k = 0; k < NSLOT - 1; k++)
		issue(k);
	for (int k = 0; k < nblk; k++) {
		if (k + NSLOT - 1 < nblk)
			issue(k + NSLOT - 1);
		/* slot k's 8 DMAs retired: the (NSLOT - 1) younger slots' 8 DMAs each may stay in flight */
		const unsigned sl = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned *)(ring + (k % NSLOT) * M * 64 + lane);
		unsigned v[M];
		if (k + NSLOT - 1 < nblk) {
			if (NSLOT == 2)
				asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
			else if (NSLOT == 3)
				asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
			else
				asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
		} else {
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		}
#pragma unroll
		for (int m = 0; m < M; m++)
			asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v[m]) : "v"(sl), "i"(m * 256) : "memory");
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
		for (int m = 0; m < M; m++)
			acc ^= v[m];
		if (t == check_tile && k == 0) {	/* correctness: frames 0..7 of wave 0's first block */
#pragma unroll
			for (int m = 0; m < M; m++)
				out[64 + ((wave * M + m) * 64 + lane)] = v[m];
		}
		/* the slot is rewritten NSLOT - 1 blocks later: the reads above have completed (lgkmcnt 0) */
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

template <int NSLOT>
static void run_lds(const char *d, const int *c1, unsigned *o, size_t lds_extra, const char *what) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const int ntiles = H * (W * 2 / 256);
	const size_t lds = (size_t)4 * NSLOT * 8 * 256 + lds_extra;
	auto kf = k_probe_lds<NSLOT>;
	(void)hipFuncSetAttribute((const void *)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
	hipLaunchKernelGGL(kf, dim3(ntiles), dim3(256), lds, 0, d, c1, o, ntiles, 12345);
	(void)hipDeviceSynchronize();
	(void)hipEventRecord(a);
	for (int i = 0; i < 5; i++)
		hipLaunchKernelGGL(kf, dim3(ntiles), dim3(256), lds, 0, d, c1, o, ntiles, -1);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 5;
	int per_cu = 0;
	(void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kf, 256, lds);
	printf("LDS-DMA NSLOT=%d lds=%6zu (%s) wg/cu=%d: %7.3f ms %7.1f GB/s (%s)\n", NSLOT, lds, what, per_cu, ms,
			(double)NF * FRAMEB / ms / 1e6, hipGetErrorString(hipGetLastError()));
	fflush(stdout);
}

/* the LDS-DMA data of the check tile (12345, frames 0..31 of its waves' first blocks) against the
 * bytes the frames hold at the shifted (2-byte aligned) addresses */
static int check_lds(const char *d, const int *h_c1, unsigned *o) {
	const int ntx = (W * 2) / 256, per_xcd = H * ntx / 8;
	/* invert the XCD-major deal: blockIdx b -> tile xcd * per_xcd + (b >> 3) */
	const int t = 12345, xt = t % ntx, R = t / ntx;
	static unsigned got[4 * 8 * 64];
	(void)hipMemcpy(got, o + 64, sizeof got, hipMemcpyDeviceToHost);
	(void)per_xcd;
	int bad = 0, odd = 0;
	for (int wave = 0; wave < 4; wave++)
		for (int m = 0; m < 8; m++) {
			const int f = wave * 8 + m;
			const long so = (long)R * W * 2 + xt * 256 + h_c1[f];
			odd += (so & 3) != 0;
			unsigned char bytes[260];
			const long lo = so < 0 ? 0 : so;
			(void)hipMemcpy(bytes, d + (size_t)f * FRAMEB + lo, 260, hipMemcpyDeviceToHost);
			for (int lane = 0; lane < 64; lane++) {
				const long a = so + lane * 4;
				unsigned want = 0;
				if (a >= 0 && a + 4 <= (long)FRAMEB)
					memcpy(&want, bytes + (a - lo), 4);
				if (got[(wave * 8 + m) * 64 + lane] != want && bad++ < 5)
					printf("  mismatch frame %d lane %d (src offset %ld): got %08x want %08x\n", f, lane, a,
							got[(wave * 8 + m) * 64 + lane], want);
			}
		}
	printf("LDS-DMA data check: %d of %d dwords differ (%d of 32 frames at a 2-byte-misaligned source)\n", bad,
			4 * 8 * 64, odd);
	return bad;
}

__global__ void k_fill(unsigned *p, size_t n) {
	for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		p[i] = (unsigned)(i * 2654435761u);
}

template <int TW, int LW, int NBUF, bool PERSIST, int M = 16>
static void run(const char *d, const int *c1, unsigned *o, int waves, int wg_per_cu, size_t lds) {
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	const int ntiles = H * (W * 2 / TW);
	const int grid = PERSIST ? 256 * wg_per_cu : ntiles;
	auto kf = k_probe<TW, LW, NBUF, PERSIST, M>;
	(void)hipFuncSetAttribute((const void *)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
	hipLaunchKernelGGL(kf, dim3(grid), dim3(64 * waves), lds, 0, d, c1, o, ntiles);
	(void)hipDeviceSynchronize();
	(void)hipEventRecord(a);
	for (int i = 0; i < 5; i++)
		hipLaunchKernelGGL(kf, dim3(grid), dim3(64 * waves), lds, 0, d, c1, o, ntiles);
	(void)hipEventRecord(b);
	(void)hipEventSynchronize(b);
	float ms;
	(void)hipEventElapsedTime(&ms, a, b);
	ms /= 5;
	printf("M=%2d TW=%4d LW=%2d NBUF=%d %s waves=%2d wg/cu=%d lds=%6zu: %7.3f ms %7.1f GB/s (%s)\n", M, TW, LW, NBUF,
			PERSIST ? "persist" : "tiles  ", waves, wg_per_cu, lds, ms, (double)NF * FRAMEB / ms / 1e6,
			hipGetErrorString(hipGetLastError()));
	fflush(stdout);
}

int main(int argc, char **argv) {
	char *d;
	unsigned *o;
	int *c1;
	if (hipMalloc(&d, (size_t)NF * FRAMEB) != hipSuccess) {
		printf("alloc failed\n");
		return 1;
	}
	(void)hipMalloc(&o, 65536);	/* out[0] + the LDS-DMA check block (out[64 .. 64 + 2048)) */
	(void)hipMalloc(&c1, NF * sizeof(int));
	int h[NF];
	const int zero = argc > 1 && atoi(argv[1]) == 0;
	for (int f = 0; f < NF; f++) {
		int sx = 0, sy = 0;
		if (f && !zero) {
			const uint64_t z = mix64(0x5151ull ^ 0x51B1ull ^ ((uint64_t)f << 32));
			sx = -((int)((z & 0xFFFFFFFFu) % 33) - 16);
			sy = -((int)(((z >> 32) & 0xFFFFFFFFu) % 33) - 16);
		}
		h[f] = -(sy * W * 2 + 2 * sx);
	}
	(void)hipMemcpy(c1, h, sizeof h, hipMemcpyHostToDevice);
	hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, (unsigned *)d, (size_t)NF * FRAMEB / 4);
	(void)hipDeviceSynchronize();
	const int mode = argc > 2 ? atoi(argv[2]) : 0;
	if (mode == 6) {
		run_lds<2>(d, c1, o, 0, "ring only");
		if (check_lds(d, h, o))
			return 1;
		for (int rep = 0; rep < 2; rep++) {
			run<256, 4, 2, false>(d, c1, o, 4, 4, 34560);	/* today's register-staged geometry */
			run<256, 4, 2, false, 8>(d, c1, o, 4, 4, 34560);
			run_lds<2>(d, c1, o, 0, "ring only");
			run_lds<2>(d, c1, o, 24000, "ring + 24 KB");
			run_lds<2>(d, c1, o, 34560, "ring + histogram");
			run_lds<3>(d, c1, o, 0, "ring only");
			run_lds<3>(d, c1, o, 14000, "ring + 14 KB");
			run_lds<4>(d, c1, o, 0, "ring only");
		}
		return 0;
	}
	if (mode == 5) {	/* round 5: 512-B segments at 3 or 4 workgroups per CU */
		for (int rep = 0; rep < 2; rep++) {
			run<256, 4, 2, false>(d, c1, o, 4, 4, 34560);		/* today's geometry */
			run<512, 4, 2, false, 8>(d, c1, o, 4, 3, 50000);
			run<512, 4, 2, false>(d, c1, o, 4, 3, 50000);
			run<512, 4, 2, false, 8>(d, c1, o, 8, 3, 50000);
			run<512, 4, 2, false>(d, c1, o, 8, 3, 50000);
			run<512, 4, 2, false, 8>(d, c1, o, 4, 4, 36000);
			run<512, 4, 2, false>(d, c1, o, 4, 4, 36000);
			run<512, 4, 2, false, 8>(d, c1, o, 8, 2, 70000);
			run<512, 4, 2, false, 8>(d, c1, o, 4, 2, 70000);
			run<1024, 4, 2, false, 8>(d, c1, o, 8, 2, 70000);
			run<1024, 4, 2, false, 8>(d, c1, o, 4, 3, 50000);
		}
		return 0;
	}
	for (int rep = 0; rep < 2; rep++) {
		run<256, 4, 2, false>(d, c1, o, 4, 4, 34560);
		run<512, 4, 2, false>(d, c1, o, 8, 2, 70000);
		run<512, 4, 2, false, 8>(d, c1, o, 8, 2, 70000);
		run<512, 4, 3, false, 8>(d, c1, o, 8, 2, 70000);
		run<512, 4, 4, false, 8>(d, c1, o, 8, 2, 70000);
		run<512, 4, 3, false>(d, c1, o, 8, 2, 70000);
		run<512, 4, 2, false>(d, c1, o, 4, 2, 70000);
		run<512, 4, 3, false>(d, c1, o, 4, 2, 70000);
		run<512, 4, 2, false>(d, c1, o, 8, 1, 100000);
		run<1024, 4, 2, false, 8>(d, c1, o, 16, 1, 140000);
		run<1024, 4, 2, false, 8>(d, c1, o, 8, 1, 140000);
		run<1024, 4, 3, false, 8>(d, c1, o, 8, 1, 140000);
	}
	return 0;
}

/*
 * sg_api.cpp - C ABI of libsirilgpu.so (include/sirilgpu.h): contexts, HBM workspaces,
 * kernel selection and the host-pull stacking path.
 *
 * Everything here is plumbing around the gfx950 kernels of sg_stack.hip / sg_register.hip;
 * no pixel is ever computed on the host.  If a launch fails the call fails loudly
 * (SG_ERR_DEVICE + sg_last_error), there is no CPU fallback.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <vector>
#include <string>
#include <algorithm>
#include <array>
#include <atomic>
#include <mutex>
#include <thread>
#include "sg_common.hpp"
#include "../../include/sirilgpu.h"

struct SgChainTables {
	const int *blk_of_row;
	const int *blk_channel, *blk_start, *blk_end, *blk_first;
	int nblocks;
};

template <int NREG, bool LISTED>
__global__ void k_stack_sorted(SgStackParams p, const unsigned int *list, const unsigned int *list_count);
template <int REJ, int NORM, int NI>
__global__ void k_stack_hist(SgStackParams p, const int *tab, const int4 *norm, unsigned int *redo_count,
		unsigned int *redo_list);
__global__ void k_norm_fma_check(double *pairs, int N, int npad, int mode, unsigned int *verdict);
template <int KM, int NW, bool PAIR>
__global__ void k_stack_linfit(SgStackParams p, unsigned int *redo_count, unsigned int *redo_list);
__global__ void k_hist_slow(SgStackParams p, unsigned int *redo_count, unsigned int *redo_list);
void sg_dbg_why_dump(hipStream_t s);
int sgh_block_threads(int ni, int rej);
template <int NM>
__global__ void k_stack_replay(SgStackParams p);
__global__ void k_redo_to_literal(SgStackParams p, const unsigned int *list, const unsigned int *count,
		unsigned int maxn);
__global__ void k_stack_reduce(SgStackParams p);
__global__ void k_stack_reduce2(SgStackParams p);
template <int M, int SEG>
__global__ void k_stack_reduce3(SgStackParams p, const int *tab, const int *shifty);
__global__ void k_sum_finalize(SgStackParams p);
__global__ void k_stack_literal(SgStackParams p, SgChainTables t, unsigned int count, uint8_t *scratch, int phase);
__global__ void k_synth_fill(uint16_t *frames, int first_frame, int nframes, int C, int H, int W, int row_begin,
		int row_end, uint64_t seed, int maxshift, int64_t frame_stride, int64_t plane_stride);

#include "sg_ctx.hpp"

__global__ void k_flip_rows(const uint16_t *src, uint16_t *dst, int W, int rows);
__global__ void k_stage_copy(uint4 *dst, const uint4 *src, unsigned int n16);
__global__ void k_linfit_tables(double *tab, int nmax);
__global__ void k_list_all(SgStackParams p);
__global__ void k_ctr_finalize(unsigned long long *ctr, unsigned long long *host);
/* host-pull readers per device and the bytes of one region read (two pinned + two device
 * staging buffers of this size per reader) */
#define SG_PULL_READERS 8
#define SG_PULL_CHUNK_BYTES ((size_t)4 << 20)
/* rejection counter shards at the start of the counter block (SgDevice::ctr) */
static const size_t SG_CTR_REJB = sizeof(unsigned long long) * SG_REJ_SHARDS * 6;

extern "C" int sg_init(sg_ctx **out, int ndev, const int *devs) {
	if (!out)
		return SG_ERR_GENERIC;
	*out = nullptr;
	int count = 0;
	if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
		return SG_ERR_DEVICE;
	sg_ctx *ctx = new sg_ctx();
	memset(&ctx->stats, 0, sizeof ctx->stats);
	ctx->knobs.read();
	if (ndev < 0) {	/* every visible device */
		ndev = count;
		devs = nullptr;
	}
	if (ndev == 0)
		ndev = 1;
	for (int i = 0; i < ndev; i++) {
		SgDevice d;
		d.id = devs ? devs[i] : i;
		if (d.id < 0 || d.id >= count) {
			delete ctx;
			return SG_ERR_DEVICE;
		}
		if (hipSetDevice(d.id) != hipSuccess || hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess) {
			delete ctx;
			return SG_ERR_DEVICE;
		}
		for (int k = 0; k < 4; k++)
			(void)hipEventCreate(&d.ev[k]);
		for (int k = 0; k < 2; k++) {
			for (int j = 0; j < 3; j++)
				(void)hipEventCreate(&d.cev[k][j]);
			(void)hipEventCreateWithFlags(&d.sl[k].stage_ev, hipEventDisableTiming);
		}
		for (int k = 0; k < 2; k++)
			(void)hipEventCreateWithFlags(&d.io_ev[k], hipEventDisableTiming);
		ctx->dev.push_back(d);
	}
	for (auto &a : ctx->dev)
		for (auto &b : ctx->dev)
			a.shared += (&a != &b && a.id == b.id) ? 1 : 0;
	*out = ctx;
	return SG_OK;
}

extern "C" void sg_shutdown(sg_ctx *ctx) {
	if (!ctx)
		return;
	for (auto &d : ctx->dev) {
		(void)hipSetDevice(d.id);
		(void)hipStreamSynchronize(d.stream);
		if (d.tail)
			(void)hipStreamSynchronize(d.tail);
		SgBuf *bufs[] = {&d.sum_buf, &d.frames, &d.out, &d.reg_sel, &d.reg_spec, &d.reg_work, &d.reg_tw, &d.reg_tw32,
			&d.reg_best, &d.reg_qbuf, &d.reg_qacc, &d.zeros, &d.io_raw, &d.io_bad, &d.warp_tab, &d.stats_buf, &d.ctr};
		for (SgBuf *b : bufs)
			if (b->p)
				(void)hipFree(b->p);
		for (SgSlot &q : d.sl) {
			SgBuf *sb[] = {&q.inb, &q.flag_list, &q.flag_map, &q.redo, &q.cmp_cols, &q.cmp_list, &q.scratch, &q.lin_tab,
				&q.wx};
			for (SgBuf *b : sb)
				if (b->p)
					(void)hipFree(b->p);
			if (q.stage_h)
				(void)hipHostFree(q.stage_h);
			if (q.stage_ev)
				(void)hipEventDestroy(q.stage_ev);
		}
		if (d.tail)
			(void)hipStreamDestroy(d.tail);
		if (d.tail_ev)
			(void)hipEventDestroy(d.tail_ev);
		if (d.tail_done_ev)
			(void)hipEventDestroy(d.tail_done_ev);
		for (int k = 0; k < 2; k++)
			if (d.pinned[k])
				(void)hipHostFree(d.pinned[k]);
		if (d.ctr_h)
			(void)hipHostFree(d.ctr_h);
		for (int k = 0; k < 2; k++) {
			if (d.io_stage[k])
				(void)hipHostFree(d.io_stage[k]);
			if (d.io_ev[k])
				(void)hipEventDestroy(d.io_ev[k]);
		}
		for (int k = 0; k < 4; k++)
			if (d.ev[k])
				(void)hipEventDestroy(d.ev[k]);
		for (int k = 0; k < 2; k++)
			for (int j = 0; j < 3; j++)
				if (d.cev[k][j])
					(void)hipEventDestroy(d.cev[k][j]);
		for (SgReader &rd : d.readers) {
			if (rd.stream)
				(void)hipStreamSynchronize(rd.stream);
			for (int k = 0; k < 2; k++) {
				if (rd.pin[k])
					(void)hipHostFree(rd.pin[k]);
				if (rd.dstage[k])
					(void)hipFree(rd.dstage[k]);
				if (rd.ev[k])
					(void)hipEventDestroy(rd.ev[k]);
			}
			if (rd.stream)
				(void)hipStreamDestroy(rd.stream);
		}
		if (d.aux) {
			(void)hipStreamSynchronize(d.aux);
			(void)hipStreamDestroy(d.aux);
		}
		for (int k = 0; k < 2; k++)
			if (d.aux_ev[k])
				(void)hipEventDestroy(d.aux_ev[k]);
		if (d.qacc_h)
			(void)hipHostFree(d.qacc_h);
		if (d.aux2) {
			(void)hipStreamSynchronize(d.aux2);
			(void)hipStreamDestroy(d.aux2);
		}
		for (int k = 0; k < 2; k++)
			if (d.aux2_ev[k])
				(void)hipEventDestroy(d.aux2_ev[k]);
		if (d.reg_pin)
			(void)hipHostFree(d.reg_pin);
		(void)hipStreamDestroy(d.stream);
	}
	delete ctx;
}

extern "C" const char *sg_last_error(const sg_ctx *ctx) {
	return ctx ? ctx->err.c_str() : "no context";
}

extern "C" int sg_get_last_stats(const sg_ctx *ctx, sg_stack_stats *st) {
	if (!ctx || !st)
		return SG_ERR_GENERIC;
	std::lock_guard<std::mutex> lk(((sg_ctx *)ctx)->mu);
	*st = ctx->stats;
	return SG_OK;
}

extern "C" int sg_device_count(const sg_ctx *ctx, int *ndev) {
	if (!ctx || !ndev)
		return SG_ERR_GENERIC;
	*ndev = (int)ctx->dev.size();
	return SG_OK;
}

/* ---- reference block partition (src/stacking/stacking.c:1397-1476) and the libgomp
 *      schedule(static) assignment of blocks to OpenMP threads (:1513-1516) ---- */
struct Block {
	long channel, start_row, end_row;
};

static int make_blocks(long H, int nb_channels, int max_number_of_rows, int nb_threads,
		std::vector<Block> &blocks) {
	int size_of_stacks = max_number_of_rows / nb_threads;
	if (size_of_stacks == 0)
		size_of_stacks = 1;
	long nb_parallel_stacks;
	int remainder;
	if (H / size_of_stacks < 4) {
		nb_parallel_stacks = 4 * nb_channels;
		size_of_stacks = (int)(H / 4);
		remainder = (int)(H % 4);
	} else {
		nb_parallel_stacks = H * nb_channels / size_of_stacks;
		if (nb_parallel_stacks % nb_channels != 0 || (H * nb_channels) % size_of_stacks != 0) {
			nb_parallel_stacks += nb_channels - (nb_parallel_stacks % nb_channels);
			size_of_stacks = (int)(H * nb_channels / nb_parallel_stacks);
		}
		remainder = (int)(H - (nb_parallel_stacks / nb_channels * size_of_stacks));
	}
	if (size_of_stacks <= 0)
		return -1;
	blocks.clear();
	long channel = 0, row = 0, end;
	do {
		if ((long)blocks.size() >= nb_parallel_stacks)
			return -1;
		Block b;
		b.channel = channel;
		b.start_row = row;
		end = row + size_of_stacks - 1;
		if (remainder > 0) {
			end++;
			remainder--;
		}
		if (end >= H - 1 || (H - end < size_of_stacks / 10)) {
			end = H - 1;
			row = 0;
			channel++;
			remainder = (int)(H - (nb_parallel_stacks / nb_channels * size_of_stacks));
		} else {
			row = end + 1;
		}
		b.end_row = end;
		blocks.push_back(b);
	} while (channel < nb_channels);
	return (long)blocks.size() == nb_parallel_stacks ? 0 : -1;
}

static void omp_static_chunk(long n, int nthr, int t, long *begin, long *end) {
	long q = n / nthr, r = n % nthr;
	if (t < r) {
		q++;
		*begin = q * t;
	} else {
		*begin = q * t + r;
	}
	*end = *begin + q;
}

static int default_threads(void) {
	long n = sysconf(_SC_NPROCESSORS_ONLN);
	return n > 0 ? (int)n : 1;
}

static int pick_nreg(int N) {
	if (N <= 64) return 1;
	if (N <= 128) return 2;
	if (N <= 256) return 4;
	if (N <= 512) return 8;
	if (N <= 1024) return 16;
	return 0;
}

static hipError_t launch_sorted(int nreg, bool listed, dim3 grid, size_t lds, hipStream_t s, const SgStackParams &p,
		const unsigned int *list, const unsigned int *list_count) {
	switch (nreg * 2 + (listed ? 1 : 0)) {
#define SG_CASE(R, LI)                                                                              \
	case R * 2 + LI:                                                                            \
		(void)hipFuncSetAttribute((const void *)k_stack_sorted<R, LI>,                      \
				hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);              \
		hipLaunchKernelGGL((k_stack_sorted<R, LI>), grid, dim3(SG_SORT_THREADS), lds, s, p, list,  \
				list_count);                                                        \
		return hipGetLastError();
		SG_CASE(1, 0)
		SG_CASE(1, 1)
		SG_CASE(2, 0)
		SG_CASE(2, 1)
		SG_CASE(4, 0)
		SG_CASE(4, 1)
		SG_CASE(8, 0)
		SG_CASE(8, 1)
		SG_CASE(16, 0)
		SG_CASE(16, 1)
#undef SG_CASE
	}
	return hipErrorInvalidValue;
}

/* k_stack_literal: one thread per queued pixel with N * 5 bytes of scratch each; SG_LIT_THREADS
 * threads up to 2048 frames, then as many as 1 GiB of scratch holds (at least 4096) */
static unsigned lit_thread_count(int N) {
	const size_t lit_bytes = ((size_t)N * 5 + 15) & ~(size_t)15;
	return (unsigned)std::max<size_t>(4096, std::min<size_t>(SG_LIT_THREADS, ((size_t)1 << 30) / lit_bytes) & ~(size_t)63);
}
static size_t lit_scratch_bytes(int N) {
	return (size_t)lit_thread_count(N) * (((size_t)N * 5 + 15) & ~(size_t)15);
}

/* SUM over row bands streamed by the host-pull path: the raw sums and the maximum carry
 * across the band calls, the scaling runs once after the last band */
enum { SUM_WHOLE = 0, SUM_FIRST_BAND = 1, SUM_MID_BAND = 2, SUM_LAST_BAND = 3 };

/* counter block of one slot: rejection shards, then {flag count, walk fault, redo count, compact
 * count, loop fault} and the SUM maximum 64 bytes further */
static const size_t SG_CTRB = SG_CTR_REJB + 128;
/* host-mapped slot k_ctr_finalize writes: rejection sums at 0, the flag block at 64 */
static const size_t SG_CTR_HOSTB = 256;
/* blocks of the listed k_stack_sorted launches (grid-stride over any list length) */
#define SG_LIST_GRID 1024

/*
 * wait for the call queued in counter slot `slot` and take its results: faults, the rejection
 * counters (rej, may be null), the SUM maximum, the call's statistics (published to the context)
 */
static int stack_fold(sg_ctx *ctx, SgDevice &dv, int slot, uint64_t rej[3][2], uint64_t *maxim_out, bool sync) {
	HIPCHK(hipEventSynchronize(dv.cev[slot][2]));
	dv.pend[slot] = false;
	dv.sl[slot].stage_pending = false;	/* the input copy ran before this call's kernels */
	const char *h = (const char *)dv.ctr_h + (size_t)slot * SG_CTR_HOSTB;
	const unsigned int *fl = (const unsigned int *)(h + 64);
	sg_stack_stats &st = dv.pstats[slot];
	float ms = 0.f, ms2 = 0.f;
	HIPCHK(hipEventElapsedTime(&ms, dv.cev[slot][0], dv.cev[slot][1]));
	HIPCHK(hipEventElapsedTime(&ms2, dv.cev[slot][0], dv.cev[slot][2]));
	st.kernel_ms = ms;
	st.total_ms = ms2;
	st.slow_pixels = fl[0];
	if (st.path == 1)
		st.chain_pixels = fl[2];
	st.compact_pixels = std::min<uint64_t>(fl[3], st.compact_pixels);	/* pstats holds the capacity */
	st.exported_pixels = st.exported_pixels ? std::min<uint64_t>(fl[6], st.exported_pixels) : 0;	/* capacity, as compact */
	if (st.norm_fma > 0)	/* k_norm_fma_check's verdict, read back beside the counters (the launch set the best allowed) */
		st.norm_fma = st.norm_fma == 2 && !(fl[7] & 2u) ? 2 : (fl[7] & 1u) ? 0 : 1;
	if (sync) {	/* the calling stack_device_core publishes dv.stats when it returns */
		dv.stats = st;
	} else {
		std::lock_guard<std::mutex> lk(ctx->mu);
		ctx->stats = st;
	}
	if (fl[4])
		return set_err(ctx, SG_ERR_GENERIC, "SIGMEDIAN: the reference's clipping loop never ends for some pixel "
				"(a pass replaces samples by the values they already hold, stacking.c:1696-1709)%s%.0ld", "", 0);
	if (fl[1])
		return set_err(ctx, SG_ERR_WALK, "a first-pass early break needs the stale rejected[] of a pixel "
				"whose frame rows are not resident; make the full frames resident%s%.0ld", "", 0);
	if (rej) {
		const unsigned long long *sums = (const unsigned long long *)h;	/* k_ctr_finalize's */
		for (int c = 0; c < 3; c++) {
			rej[c][0] = sums[c * 2];
			rej[c][1] = sums[c * 2 + 1];
		}
	}
	if (maxim_out)
		*maxim_out = dv.pend_sum_read[slot] ? fl[16] : 0;
	return SG_OK;
}

/* fold a pending async call into the device's accumulators (sg_stack_collect returns them) */
static void stack_fold_acc(sg_ctx *ctx, SgDevice &dv, int slot) {
	uint64_t r[3][2], mx = 0;
	const int rc = stack_fold(ctx, dv, slot, r, &mx, false);
	if (rc) {
		if (!dv.acc_rc)
			dv.acc_rc = rc == SG_ERR_WALK ? SG_ERR_GENERIC : rc;
		return;
	}
	for (int c = 0; c < 3; c++) {
		dv.acc_rej[c][0] += r[c][0];
		dv.acc_rej[c][1] += r[c][1];
	}
	dv.acc_max = std::max<uint64_t>(dv.acc_max, mx);
}

static int stack_device_core(sg_ctx *ctx, int dev_index, const sg_stack_desc *d,
		const uint16_t *d_frames, int64_t frame_stride, int64_t plane_stride, uint16_t *d_out,
		int row_begin, int row_end, uint64_t rej[3][2], uint64_t *maxim_out, void *stream, int sum_mode,
		bool async = false, int *slot_out = nullptr) {
	if (!ctx || !d || dev_index < 0 || dev_index >= (int)ctx->dev.size())
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[dev_index];
	const int N = d->nb_frames, W = d->width, H = d->height, C = d->nb_layers;
	if (N < 2)
		return set_err(ctx, SG_ERR_GENERIC, "select at least two frames (%s%ld)", "", N);
	if (W <= 0 || H <= 0 || C < 1 || C > 3 || row_begin < 0 || row_end > H || row_begin >= row_end)
		return set_err(ctx, SG_ERR_SIZE, "bad geometry%s %ld", "", 0);
	if (d->method < 0 || d->method > 4)
		return set_err(ctx, SG_ERR_GENERIC, "unknown method%s %ld", "", d->method);
	HIPCHK(hipSetDevice(dv.id));
	hipStream_t s = stream ? (hipStream_t)stream : dv.stream;
	const int nrows = row_end - row_begin;
	const size_t npix_img = (size_t)C * H * W;
	/* this call's statistics: the device's own record (one thread per device), published to the
	 * context when the call returns, whatever the outcome */
	sg_stack_stats &st = dv.stats;
	memset(&st, 0, sizeof st);
	struct Publish {
		sg_ctx *c;
		const sg_stack_stats &s;
		bool on;
		~Publish() {
			if (!on)	/* an async call's statistics are published when it is folded */
				return;
			std::lock_guard<std::mutex> lk(c->mu);
			c->stats = s;
		}
	} publish{ctx, st, !async};

	SgStackParams p;
	memset(&p, 0, sizeof p);
	p.frames = d_frames;
	p.frame_stride = frame_stride;
	p.plane_stride = plane_stride;
	p.out = d_out;
	p.N = N;
	p.W = W;
	p.H = H;
	p.C = C;
	p.method = d->method;
	p.rejection = d->rejection;
	p.normalize = (d->method == SG_STACK_MEAN || d->method == SG_STACK_MEDIAN) ? d->normalize : 0;
	p.sig0 = d->sig[0];
	p.sig1 = d->sig[1];
	p.use_shift = (d->method != SG_STACK_MEDIAN) && d->shiftx && d->shifty;
	p.row_begin = row_begin;
	p.row_end = row_end;
	p.res_begin = 0;
	p.res_end = H;
	if (d->resident_rows[0] != 0 || d->resident_rows[1] != 0) {
		p.res_begin = d->resident_rows[0];
		p.res_end = d->resident_rows[1];
		if (p.res_begin < 0 || p.res_end > H || p.res_begin >= p.res_end)
			return set_err(ctx, SG_ERR_SIZE, "bad resident row range%s %ld", "", (long)p.res_begin);
	}
	p.sy_min = p.sy_max = 0;
	if (p.use_shift) {
		p.sy_min = p.sy_max = d->shifty[0];
		for (int i = 1; i < N; i++) {
			p.sy_min = std::min(p.sy_min, d->shifty[i]);
			p.sy_max = std::max(p.sy_max, d->shifty[i]);
		}
	}
	{
		/* the frame rows the band's output rows read (R - shifty, :1550-1577) must be resident */
		const int lo = (int)std::max<int64_t>(0, (int64_t)row_begin - p.sy_max);
		const int hi = (int)std::min<int64_t>(H - 1, (int64_t)row_end - 1 - p.sy_min);
		if (lo <= hi && (lo < p.res_begin || hi >= p.res_end)) {
			char m[160];
			snprintf(m, sizeof m, "frame rows %d..%d read by the band are not all resident (%d..%d)", lo, hi,
					p.res_begin, p.res_end - 1);
			return set_err(ctx, SG_ERR_SIZE, "%s%.0ld", m, 0);
		}
	}
	p.dbg = ctx->knobs.hist_dbg;
	p.prio = ctx->knobs.hist_prio;	/* 1 measured best: 4.73 -> 4.58 ms (scripts/gpu_prio.sh) */
	p.wins_cap = ctx->knobs.wins_cap;

	/* per-frame constants: shifts + normalisation coefficients */
	const int Npad = (N + 15) & ~15;	/* histogram-path table: 64-byte aligned, padded */
	/* layout: c1[Npad] int, sx2[Npad] int16, shiftx[N], shifty[N]; the call's inputs (this
	 * table, the normalisation coefficients, the chain tables) reach the device in one copy
	 * (flush_inputs, right before the first kernel) */
	std::vector<int> sh(Npad + Npad / 2 + 2 * N, 0);
	std::vector<double> nm;
	std::vector<int> tables, ztab;
	/* the histogram path addresses a frame plane with 32-bit offsets: (R - sy) W 2 must fit */
	bool hist_addr_ok = (int64_t)H * W * 2 <= (1ll << 30);
	{
		/* per frame c1 = shifty*W*2 + 2*shiftx and sx2 = 2*shiftx for the histogram path
		 * (zeros when there is no registration data), then the plain shift arrays */
		int16_t *sx2 = (int16_t *)(sh.data() + Npad);
		p.hist_maxsx = 0;
		for (int i = 0; p.use_shift && i < N; i++) {
			const int64_t sy = d->shifty[i], sx = d->shiftx[i];
			const int64_t asy = sy < 0 ? -sy : sy, asx = sx < 0 ? -sx : sx;
			if ((int64_t)(H + asy) * W * 2 + 2 * asx >= (1ll << 31) || asx > 16383)
				hist_addr_ok = false;
			sh[i] = (int)(sy * W * 2 + 2 * sx);
			sx2[i] = (int16_t)(2 * sx);
			if (asx > p.hist_maxsx)
				p.hist_maxsx = (int)asx;
		}
		if (p.use_shift) {
			memcpy(sh.data() + Npad + Npad / 2, d->shiftx, sizeof(int) * N);
			memcpy(sh.data() + Npad + Npad / 2 + N, d->shifty, sizeof(int) * N);
		}
	}
	if (p.normalize) {
		nm.resize(3 * N);
		for (int i = 0; i < N; i++) {
			nm[i] = d->offset ? d->offset[i] : 0.0;
			nm[N + i] = d->mul ? d->mul[i] : 1.0;
			nm[2 * N + i] = d->scale ? d->scale[i] : 1.0;
		}
		/* the histogram path's per-frame pair {scale, offset} (additive) or {scale, mul}
		 * (multiplicative), read with one scalar load per frame */
		const bool additive = p.normalize == SG_ADDITIVE || p.normalize == SG_ADDITIVE_SCALING;
		/* + Npad single-rounding candidate pairs and the flag word of k_norm_fma_check (bit 0: no fma
		 * load, bit 1: no integer load; the check ORs in what it finds) */
		nm.resize(3 * N + 6 * Npad + 2, 0.0);	/* + the integer offsets of k_norm_fma_check's scale-1 form */
		{
			/* SG_NORM_FMA 0: neither form, 1: the fma only, 2 (default): the integer form first */
			const unsigned int staged = ctx->knobs.norm_fma == 0 ? 3u : (ctx->knobs.norm_fma == 1 ? 2u : 0u);
			memcpy(&nm[3 * N + 4 * Npad], &staged, sizeof staged);
		}
		/* additive: when every offset - 0.5 is exact (TwoSum error 0), the pair carries
		 * offset - 0.5 and the kernel folds round_to_WORD's + 0.5 into the subtraction
		 * (NORM 3: trunc(v scale - (offset - 0.5)), one fp64 add per sample less; equal to
		 * trunc((v scale - offset) + 0.5) whenever the fold is exact, tests/test_norm_fold.py) */
		bool fold = additive;
		for (int i = 0; fold && i < N; i++) {
			const double b = nm[i], c = b - 0.5, bb = c - b;
			fold = ((b - (c - bb)) + (-0.5 - bb)) == 0.0;
		}
		p.hist_norm_fold = fold ? 1 : 0;
		for (int i = 0; i < N; i++) {
			nm[3 * N + 2 * i] = nm[2 * N + i];
			nm[3 * N + 2 * i + 1] = additive ? (fold ? nm[i] - 0.5 : nm[i]) : nm[N + i];
		}
	}
	/* additive normalisation with shifts: a row whose shifted source row leaves frame f holds
	 * f's normalised zero round_to_WORD(0 scale - offset) (:1550-1577 zero fill, then
	 * :1635-1652); the histogram path takes those values per border row from this table
	 * (SghPix::zmax) instead of sending the rows to the redo list */
	if (p.use_shift && (p.normalize == SG_ADDITIVE || p.normalize == SG_ADDITIVE_SCALING)) {
		int k1 = std::max(0, p.sy_max), k2 = std::max(0, -p.sy_min);
		if (k1 + k2 >= H) {
			k1 = H;
			k2 = 0;
		}
		ztab.assign((size_t)8 * (k1 + k2), 0);
		bool any = false;
		for (int t = 0; t < k1 + k2; t++) {
			const int R = t < k1 ? t : H - k2 + (t - k1);
			int zc = 0, zmin = 65535, zmax = 0;
			long long zs = 0, zss = 0;	/* 64-bit: N up to 65535 normalised zeros up to 65534 */
			for (int f = 0; f < N; f++) {
				const int sr = R - d->shifty[f];
				if (sr >= 0 && sr < H)
					continue;
				const double x = 0.0 * nm[2 * N + f] - nm[f];	/* v scale - offset at v = 0 */
				const int z = x <= 0.0 ? 0 : (x > 65535.0 ? 65535 : (int)(x + 0.5));
				if (z == 0 || z == 65535)
					continue;
				zc++;
				zs += z;
				zss += (long long)z * z;
				zmin = std::min(zmin, z);
				zmax = std::max(zmax, z);
			}
			if (!zc)
				continue;
			any = true;
			int *e = &ztab[(size_t)8 * t];
			e[0] = zc;
			e[1] = (int)(uint32_t)(zs & 0xFFFFFFFFll);
			e[6] = (int)(zs >> 32);
			e[2] = (int)(uint32_t)(zss & 0xFFFFFFFFll);
			e[3] = (int)(zss >> 32);
			e[4] = zmin;
			e[5] = zmax;
		}
		if (any) {
			p.ztab_k1 = k1;
			p.ztab_k2 = k2;
		} else {
			ztab.clear();
		}
	}
	SgChainTables ct;
	memset(&ct, 0, sizeof ct);
	/* the counter slot (and its buffers): a synchronous call uses slot 0, an async call the free
	 * slot, folding the older pending call when both are taken */
	int slot = 0;
	if (async) {
		if (dv.pend[0] && dv.pend[1])
			stack_fold_acc(ctx, dv, dv.pend_seq[0] < dv.pend_seq[1] ? 0 : 1);
		slot = dv.pend[0] ? 1 : 0;
	} else if (dv.pend[0]) {
		stack_fold_acc(ctx, dv, 0);
	}
	SgSlot &sb = dv.sl[slot];
	/* one pinned host block -> one device block; sets the kernels' pointers into it */
	auto flush_inputs = [&]() -> int {
		const size_t b_sh = sizeof(int) * sh.size(), o_nm = (b_sh + 255) & ~(size_t)255;
		const size_t b_nm = sizeof(double) * nm.size(), o_tb = (o_nm + b_nm + 255) & ~(size_t)255;
		const size_t o_zt = (o_tb + sizeof(int) * tables.size() + 255) & ~(size_t)255;
		const size_t tot = (o_zt + sizeof(int) * ztab.size() + 15) & ~(size_t)15;
		if (sb.stage_pending) {	/* an earlier call's copy may still read the host block */
			HIPCHK(hipEventSynchronize(sb.stage_ev));
			sb.stage_pending = false;
		}
		if (sb.stage_h_size < tot) {
			if (sb.stage_h)
				(void)hipHostFree(sb.stage_h);
			sb.stage_h = nullptr;
			sb.stage_h_size = 0;
			/* coherent: the device reads it uncached, so no call sees an earlier call's inputs */
			HIPCHK(hipHostMalloc(&sb.stage_h, tot, hipHostMallocMapped | hipHostMallocCoherent));
			sb.stage_h_size = tot;
			HIPCHK(hipHostGetDevicePointer(&sb.stage_d, sb.stage_h, 0));
		}
		HIPCHK(ensure(sb.inb, tot));
		char *hb = (char *)sb.stage_h;
		memcpy(hb, sh.data(), b_sh);
		if (b_nm)
			memcpy(hb + o_nm, nm.data(), b_nm);
		if (!tables.empty())
			memcpy(hb + o_tb, tables.data(), sizeof(int) * tables.size());
		if (!ztab.empty())
			memcpy(hb + o_zt, ztab.data(), sizeof(int) * ztab.size());
		hipLaunchKernelGGL(k_stage_copy, dim3((unsigned)std::min<size_t>(64, (tot / 16 + 255) / 256)), dim3(256), 0, s,
				(uint4 *)sb.inb.p, (const uint4 *)sb.stage_d, (unsigned int)(tot / 16));
		HIPCHK(hipGetLastError());
		HIPCHK(hipEventRecord(sb.stage_ev, s));
		sb.stage_pending = true;
		const char *db = (const char *)sb.inb.p;
		p.hist_tab = (const int *)db;
		p.hist_npad = Npad;
		if (p.use_shift) {
			p.shiftx = p.hist_tab + Npad + Npad / 2;
			p.shifty = p.shiftx + N;
		}
		if (p.normalize) {
			p.offset = (const double *)(db + o_nm);
			p.mul = p.offset + N;
			p.scale = p.offset + 2 * N;
			p.hist_norm = p.offset + 3 * N;
		}
		p.ztab = ztab.empty() ? nullptr : (const int *)(db + o_zt);
		if (!tables.empty()) {
			const int *tb = (const int *)(db + o_tb);
			ct.blk_of_row = tb;
			ct.blk_channel = tb + (size_t)C * H;
			ct.blk_start = ct.blk_channel + ct.nblocks;
			ct.blk_end = ct.blk_start + ct.nblocks;
			ct.blk_first = ct.blk_end + ct.nblocks;
		}
		return SG_OK;
	};
	/* counters: rejection shards, then {flag count, walk fault, redo count, compact count, loop
	 * fault} and the sum maximum 64 bytes further (kept across the bands of a streamed SUM); one
	 * memset, one read-back.  A synchronous call uses slot 0 (a streamed SUM keeps its maximum
	 * there); an async call the free slot, folding the older pending call when both are taken */
	const size_t REJB = SG_CTR_REJB, CTRB = SG_CTRB;
	{
		const void *old_ctr = dv.ctr.p;
		HIPCHK(ensure(dv.ctr, 2 * CTRB));
		if (dv.ctr.p != old_ctr)
			dv.ctr_clean[0] = dv.ctr_clean[1] = false;
	}
	if (!dv.ctr_h) {
		HIPCHK(hipHostMalloc(&dv.ctr_h, 2 * SG_CTR_HOSTB, hipHostMallocMapped | hipHostMallocCoherent));
		HIPCHK(hipHostGetDevicePointer((void **)&dv.ctr_hd, dv.ctr_h, 0));
	}
	char *cblk = (char *)dv.ctr.p + (size_t)slot * CTRB;
	hipEvent_t *cev = dv.cev[slot];
	/* the counters are zero when the slot's last call finished (k_ctr_finalize); a fresh or
	 * failed slot is cleared here (SUM keeps its maximum across the bands of a streamed sum) */
	const bool clear_max = sum_mode == SUM_WHOLE || sum_mode == SUM_FIRST_BAND;
	if (!dv.ctr_clean[slot])
		HIPCHK(hipMemsetAsync(cblk, 0, clear_max ? CTRB : REJB + 64, s));
	else if (clear_max && d->method == SG_STACK_SUM)
		HIPCHK(hipMemsetAsync(cblk + REJB + 64, 0, sizeof(unsigned int), s));
	dv.ctr_clean[slot] = false;
	p.rej = (unsigned long long *)cblk;
	p.flag_count = (unsigned int *)(cblk + REJB);
	p.walk_fault = p.flag_count + 1;
	p.loop_fault = p.flag_count + 4;
	p.maxim = (unsigned int *)(cblk + REJB + 64);

	/* stack_mean_with_rejection reads a block's rows with area.y += shifty; when a block that
	 * does not start at the top (area.y > 0) is shifted partly above the frame (area.y + shifty
	 * < 0 <= area.y + h - 1 + shifty) it places the rows it reads at offset W (area.y - shifty)
	 * instead of W (-area.y - shifty) (src/stacking/stacking.c:1555-1561): the rows land 2 area.y
	 * too low and run 2 area.y + h - largest_block_h rows past its block buffer, always a heap
	 * overflow (the neighbouring buffer or the allocator's data).  No defined result exists to
	 * reproduce, so the call refuses the shifts instead of zero filling silently */
	if (d->method == SG_STACK_MEAN && p.use_shift && p.sy_min < 0) {
		const int nthr = d->max_thread > 0 ? d->max_thread : default_threads();
		const int maxrows = d->max_number_of_rows > 0 ? d->max_number_of_rows : H;
		std::vector<Block> blocks;
		if (make_blocks(H, C, maxrows, nthr, blocks) == 0)
			for (const Block &b : blocks) {
				const long ay = b.start_row, ah = b.end_row - b.start_row + 1;
				if (ay > 0 && ay + p.sy_min < 0 && ay + ah - 1 + p.sy_max >= 0) {
					bool hit = false;
					for (int i = 0; i < N && !hit; i++)
						hit = ay + d->shifty[i] < 0 && ay + ah - 1 + d->shifty[i] >= 0;
					if (hit) {
						char m[320];
						snprintf(m, sizeof m, "a registration shift of %d rows reaches above the block starting at "
								"row %ld: the reference overflows its block buffer there (stacking.c:1555-1561); "
								"use more rows per block (max_number_of_rows / fewer threads)", p.sy_min, ay);
						return set_err(ctx, SG_ERR_GENERIC, "%s%.0ld", m, 0);
					}
				}
			}
	}
	const bool sorted = (d->method == SG_STACK_MEDIAN) ||
		(d->method == SG_STACK_MEAN && d->rejection != SG_NO_REJEC);
	/* everything after the main kernel runs on ts: the call's stream, or the device's tail stream
	 * for an async call whose result is wanted at sg_stack_collect only (it then overlaps the
	 * next call's main kernel, which uses the other slot's buffers) */
	hipStream_t ts = s;
	auto to_tail = [&]() -> int {
		if (!(async && (d->flags & SG_STACK_RESULT_AT_COLLECT)))
			return SG_OK;
		if (!dv.tail) {
			HIPCHK(hipStreamCreateWithFlags(&dv.tail, hipStreamNonBlocking));
			HIPCHK(hipEventCreateWithFlags(&dv.tail_ev, hipEventDisableTiming));
			HIPCHK(hipEventCreateWithFlags(&dv.tail_done_ev, hipEventDisableTiming));
		}
		HIPCHK(hipEventRecord(dv.tail_ev, s));
		HIPCHK(hipStreamWaitEvent(dv.tail, dv.tail_ev, 0));
		ts = dv.tail;
		return SG_OK;
	};
	if (sorted) {
		const int nreg = pick_nreg(N);
		/* histogram fast path (sg_stack_hist.hip): SIGMA / WINSORIZED / PERCENTILE rejection and
		 * stack_median, any normalisation, 16 <= N <= 65535 (per-lane zero / 65535 counters are
		 * 16-bit halves) */
		/* LINEARFIT's decision-exact kernel (k_stack_linfit, sg_stack.hip) takes the histogram
		 * path's place: its redo list goes to the sorted kernel's exact replay the same way */
		const bool linfit_fast = d->kernel_path != SG_PATH_SORTED && d->method == SG_STACK_MEAN &&
			d->rejection == SG_LINEARFIT && N >= 16 && N <= 1024 && ctx->knobs.linfit_fast;
		const bool hist = linfit_fast || (d->kernel_path != SG_PATH_SORTED && N >= 16 && N <= 65535 && hist_addr_ok &&
			(d->method == SG_STACK_MEDIAN || (d->method == SG_STACK_MEAN && (d->rejection == SG_SIGMA ||
					d->rejection == SG_WINSORIZED || d->rejection == SG_PERCENTILE ||
					(d->rejection == SG_SIGMEDIAN && ctx->knobs.hist_sigmedian)))));
		/* beyond the sorted kernel's 1024 frames only the histogram path runs; its redo pixels
		 * all go to the replay / literal kernels (they take any N) */
		/* beyond the sorted kernel's 1024 frames a stack without a histogram path (LINEARFIT, or
		 * planes past the histogram's 32-bit offsets) goes to the literal kernel pixel by pixel: slow,
		 * but any N as the reference (:1486-1507) */
		const bool literal_all = !nreg && !hist;
		const size_t npix_launch = (size_t)C * nrows * W;
		HIPCHK(ensure(sb.flag_list, sizeof(unsigned int) * npix_launch));
		{
			/* pixel classes carry this call's epoch (sg_flag_get): no per-call clear; the map is
			 * cleared when it is new or the 31 epochs wrap */
			const void *old_map = sb.flag_map.p;
			HIPCHK(ensure(sb.flag_map, npix_img));
			if (sb.flag_map.p != old_map || sb.flag_epoch <= 0 || sb.flag_epoch >= 31) {
				HIPCHK(hipMemsetAsync(sb.flag_map.p, 0, sb.flag_map.size, s));
				sb.flag_epoch = 0;
			}
			p.flag_epoch = (unsigned int)++sb.flag_epoch;
		}
		p.flag_list = (unsigned int *)sb.flag_list.p;
		p.flag_cap = (unsigned int)npix_launch;
		p.flag_map = (uint8_t *)sb.flag_map.p;

		/* reference thread order tables for the stale-state chains */
		int nthr = d->max_thread > 0 ? d->max_thread : default_threads();
		int maxrows = d->max_number_of_rows > 0 ? d->max_number_of_rows : H;
		std::vector<Block> blocks;
		if (make_blocks(H, C, maxrows, nthr, blocks))
			return set_err(ctx, SG_ERR_GENERIC, "block partition failed (the reference would read "
					"uninitialised blocks)%s%ld", "", 0);
		const int nb = (int)blocks.size();
		tables.assign((size_t)C * H + 4 * nb, 0);
		int *blk_of_row = tables.data(), *bch = blk_of_row + (size_t)C * H, *bst = bch + nb,
		    *ben = bst + nb, *bfi = ben + nb;
		for (int b = 0; b < nb; b++) {
			bch[b] = (int)blocks[b].channel;
			bst[b] = (int)blocks[b].start_row;
			ben[b] = (int)blocks[b].end_row;
			for (long r = blocks[b].start_row; r <= blocks[b].end_row; r++)
				blk_of_row[(size_t)blocks[b].channel * H + r] = b;
		}
		for (int t = 0; t < nthr; t++) {
			long b0, b1;
			omp_static_chunk(nb, nthr, t, &b0, &b1);
			for (long b = b0; b < b1; b++)
				bfi[b] = (int)b0;
		}
		ct.nblocks = nb;
		if (int rc = flush_inputs())
			return rc;

		if (d->method == SG_STACK_MEAN && p.rejection == SG_LINEARFIT) {
			HIPCHK(ensure(sb.lin_tab, sizeof(double) * 2 * ((size_t)N + 1)));
			hipLaunchKernelGGL(k_linfit_tables, dim3((N + 64) / 64), dim3(64), 0, s, (double *)sb.lin_tab.p, N);
			HIPCHK(hipGetLastError());
			p.linfit_tab = (const double *)sb.lin_tab.p;
		}
		const int ntx = (W + SG_TILE_W - 1) / SG_TILE_W;
		const size_t nblk = (size_t)ntx * nrows * C;
		/* LINEARFIT: + one rejected[] bit per frame and pixel of the tile (reject_linearfit) */
		const size_t lds = (size_t)N * SG_STAGE_STRIDE * 2 +
			(d->rejection == SG_LINEARFIT ? (size_t)64 * ((N + 31) / 32) * 4 : 0);
		if (hist) {
			HIPCHK(ensure(sb.redo, sizeof(unsigned int) * (npix_launch + 16)));
			unsigned int *redo_count = p.flag_count + 2;	/* cleared with the counters */
			unsigned int *redo_list = (unsigned int *)sb.redo.p + 16;
			HIPCHK(hipEventRecord(cev[0], s));
			/* NORM: 0 none, 1 additive (round(v scale - offset)), 2 multiplicative (round(v scale mul)),
			 * 3 additive with the folded + 0.5 */
			const int norm = p.normalize == SG_NO_NORM ? 0 :
				(p.normalize == SG_ADDITIVE || p.normalize == SG_ADDITIVE_SCALING) ? (p.hist_norm_fold ? 3 : 1) : 2;
			/* tile = 128 NI pixels of a row, 4 NI waves: NI = 1 by default (sg_stack_hist.hip);
			 * the A/B NI = 2 (SG_HIST_NI=2) exists without normalisation only (it spills there:
			 * the per-sample double arithmetic of two pixel pairs) */
			const int ni = (norm == 0 && ctx->knobs.hist_ni == 2 && (d->method == SG_STACK_MEAN &&
						(p.rejection == SG_SIGMA || p.rejection == SG_WINSORIZED))) ? 2 : 1;
			const size_t nblk_h = (size_t)((W + 128 * ni - 1) / (128 * ni)) * nrows * C;
			if (SG_DBG(p) == 14) {	/* A/B: report the resident workgroups per CU */
				int per_cu = -1;
				(void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ni == 2 ? (const void *)k_stack_hist<2, 0, 2>
						: (const void *)k_stack_hist<2, 0, 1>, sgh_block_threads(ni, 2), (size_t)ctx->knobs.hist_ldspad);
				hipDeviceProp_t prop;
				(void)hipGetDeviceProperties(&prop, dv.id);
				fprintf(stderr, "k_stack_hist: %d workgroups/CU (lds/CU %zu, lds/block max %zu, pad %d)\n", per_cu,
						(size_t)prop.maxSharedMemoryPerMultiProcessor, (size_t)prop.sharedMemPerBlock, ctx->knobs.hist_ldspad);
			}
			const size_t lds_pad = (size_t)ctx->knobs.hist_ldspad;
			/* REJ: 2 SIGMA, 4 WINSORIZED, 1 PERCENTILE, 3 SIGMEDIAN, 8 stack_median */
			const int rj = d->method == SG_STACK_MEDIAN ? 8 : p.rejection == SG_WINSORIZED ? 4 :
				p.rejection == SG_PERCENTILE ? 1 : p.rejection == SG_SIGMEDIAN ? 3 : 2;
			/* normalised SIGMA / WINSORIZED: redo pixels whose samples the tile fully knows leave
			 * their sorted columns for the sorted kernel (sgh_compact), up to a 384 MiB buffer */
			const bool compact = !linfit_fast && norm != 0 && (rj == 2 || rj == 4) && nreg && ctx->knobs.hist_compact;
			if (compact) {
				const size_t cap = std::min<size_t>(npix_launch, ctx->knobs.hist_compact >= 2 ?
						(size_t)ctx->knobs.hist_compact : ((size_t)384 << 20) / ((size_t)N * 2));
				HIPCHK(ensure(sb.cmp_cols, cap * (size_t)N * 2));
				HIPCHK(ensure(sb.cmp_list, cap * sizeof(unsigned int)));
				p.cmp_cols = (uint16_t *)sb.cmp_cols.p;
				p.cmp_list = (unsigned int *)sb.cmp_list.p;
				p.cmp_count = p.flag_count + 3;	/* cleared with the counters */
				p.cmp_cap = (unsigned int)cap;
			}
			/* WINSORIZED without normalisation: the slow columns (a zero or a 65535 sample) leave their
			 * tiles for k_hist_slow (SG_WINS_EXPORT), up to a quarter of the launch's pixels */
			const bool wexp = rj == 4 && norm == 0 && ni == 1 && !linfit_fast && ctx->knobs.wins_export;
			if (wexp) {
				const size_t cap = ((npix_launch / 4 + 63) / 64) * 64;
				HIPCHK(ensure(sb.wx, cap * (SG_HIST_HROWS + 3) * sizeof(uint32_t)));
				p.wx = (uint32_t *)sb.wx.p;
				p.wx_cap = (unsigned int)cap;
				p.wx_count = p.flag_count + 6;	/* cleared with the counters */
				p.wx_kmax = ctx->knobs.wins_export;
				st.exported_pixels = cap;	/* the capacity; clamped to the count when folded */
			}
			const dim3 hg((unsigned)nblk_h), hb((unsigned)sgh_block_threads(ni, rj));
			/* normalised: check the single-rounding load against the reference's operations over every
			 * u16 value of every frame (k_norm_fma_check, ~10 us); the kernel reads the verdict */
			if (norm != 0 && !linfit_fast) {
				if (ctx->knobs.norm_fma) {
					hipLaunchKernelGGL(k_norm_fma_check, dim3(16, (unsigned)N), dim3(256), 0, s, (double *)p.hist_norm, N, Npad,
							norm, p.flag_count + 7);
					HIPCHK(hipGetLastError());
					/* the best load allowed; the verdict replaces it when the call is folded */
					st.norm_fma = norm != 2 && ctx->knobs.norm_fma == 2 ? 2 : 1;
				}
			}
			if (linfit_fast) {
				/* one workgroup per 64 pixels of a row, the tile's columns in LDS */
				const int km = N <= 512 ? 8 : 16;
				const size_t lfx_lds = (size_t)64 * (64 * km + 2) * sizeof(uint16_t);
				/* waves per tile: 4, 8 or (KM = 8 only: 187 VGPRs at KM = 16) 16 */
				const int lw = ctx->knobs.linfit_waves;
				const int nw = lw == 4 ? 4 : (lw == 16 && km == 8) ? 16 : 8;
				/* SG_LINFIT_PAIR: both pixels of a sorted pair in lockstep (lfx_pixel2_m), 4 or 8 waves */
				const bool pr = ctx->knobs.linfit_pair && nw != 16;
				const void *kf = pr ? (km == 8 ? (nw == 4 ? (const void *)k_stack_linfit<8, 4, true> :
								(const void *)k_stack_linfit<8, 8, true>) :
							(nw == 4 ? (const void *)k_stack_linfit<16, 4, true> :
								(const void *)k_stack_linfit<16, 8, true>)) :
					km == 8 ? (nw == 4 ? (const void *)k_stack_linfit<8, 4, false> :
						nw == 8 ? (const void *)k_stack_linfit<8, 8, false> : (const void *)k_stack_linfit<8, 16, false>) :
					(nw == 4 ? (const void *)k_stack_linfit<16, 4, false> : (const void *)k_stack_linfit<16, 8, false>);
				HIPCHK(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lfx_lds));
				const dim3 lg((unsigned)((size_t)((W + 63) / 64) * nrows * C));
				void *lfx_args[] = {&p, &redo_count, &redo_list};
				HIPCHK(hipLaunchKernel(kf, lg, dim3(64 * nw), lfx_args, lfx_lds, s));
			} else
			switch ((rj == 4 ? 10 : rj == 1 ? 20 : rj == 8 ? 30 : rj == 3 ? 40 : 0) + norm +
					100 * (rj == 1 || rj == 8 || rj == 3 ? 1 : ni)) {
			case 100: hipLaunchKernelGGL((k_stack_hist<2, 0, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 101: hipLaunchKernelGGL((k_stack_hist<2, 1, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 102: hipLaunchKernelGGL((k_stack_hist<2, 2, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 103: hipLaunchKernelGGL((k_stack_hist<2, 3, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 110: hipLaunchKernelGGL((k_stack_hist<4, 0, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 111: hipLaunchKernelGGL((k_stack_hist<4, 1, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 112: hipLaunchKernelGGL((k_stack_hist<4, 2, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 113: hipLaunchKernelGGL((k_stack_hist<4, 3, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 120: hipLaunchKernelGGL((k_stack_hist<1, 0, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 121: hipLaunchKernelGGL((k_stack_hist<1, 1, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 122: hipLaunchKernelGGL((k_stack_hist<1, 2, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 123: hipLaunchKernelGGL((k_stack_hist<1, 3, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 130: hipLaunchKernelGGL((k_stack_hist<8, 0, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 131: hipLaunchKernelGGL((k_stack_hist<8, 1, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 132: hipLaunchKernelGGL((k_stack_hist<8, 2, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 133: hipLaunchKernelGGL((k_stack_hist<8, 3, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 140: hipLaunchKernelGGL((k_stack_hist<3, 0, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 141: hipLaunchKernelGGL((k_stack_hist<3, 1, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 142: hipLaunchKernelGGL((k_stack_hist<3, 2, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 143: hipLaunchKernelGGL((k_stack_hist<3, 3, 1>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 200: hipLaunchKernelGGL((k_stack_hist<2, 0, 2>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			case 210: hipLaunchKernelGGL((k_stack_hist<4, 0, 2>), hg, hb, lds_pad, s, p, p.hist_tab, (const int4 *)p.hist_norm, redo_count, redo_list); break;
			default: return set_err(ctx, SG_ERR_GENERIC, "no histogram kernel for this case%s%.0ld", "", 0);
			}
			HIPCHK(hipGetLastError());
			if (wexp) {	/* the exported columns, before anything reads the redo list */
				hipLaunchKernelGGL(k_hist_slow, dim3(3072), dim3(64), 0, s, p, redo_count, redo_list);	/* 12 waves per CU (153 VGPRs) */
				HIPCHK(hipGetLastError());
			}
			HIPCHK(hipEventRecord(cev[1], s));
			if (int rc = to_tail())
				return rc;
			st.path = 1;
			st.main_kernel_blocks = (int)nblk;
			st.launches = 1;
			st.compact_pixels = compact ? p.cmp_cap : 0;	/* the capacity; clamped to the count when folded */
			const dim3 lgrid(SG_LIST_GRID);
			if (compact) {
				/* the compact columns, any count up to the capacity (grid-stride) */
				SgStackParams q = p;
				q.cmp_src = p.cmp_cols;
				HIPCHK(launch_sorted(nreg, true, lgrid, lds, ts, q, p.cmp_list, p.cmp_count));
				st.launches++;
			}
			/* the redo pixels, routed on the device (no host round trip in the call):
			 * - SIGMA / WINSORIZED, N <= SG_REPLAY_MAXN: up to SG_REDO_REPLAY_MAX pixels straight to
			 *   the wave-per-pixel replay (every sample of a pixel gathered by one wave at once), a
			 *   longer list (rare: e.g. normalised zeros of rows near the frame border) through the
			 *   sorted kernel (measured: 22 k pixels faster in the replay, 113 k slower);
			 * - stack_median / PERCENTILE: the sorted kernel (the literal kernel's one thread per
			 *   pixel sorts slowly: 740 pixels took 8 ms);
			 * - N > 1024 (no sorted kernel): every redo pixel to the replay / literal kernels */
			const bool replay_route = nreg && d->method == SG_STACK_MEAN && (p.rejection == SG_SIGMA ||
					p.rejection == SG_WINSORIZED) && N <= SG_REPLAY_MAXN && ctx->knobs.redo_replay;
			if (replay_route) {
				SgStackParams q = p;
				q.list_minn = SG_REDO_REPLAY_MAX;	/* idle unless the list is longer */
				HIPCHK(launch_sorted(nreg, true, lgrid, lds, ts, q, redo_list, redo_count));
				p.rp_list = redo_list;
				p.rp_count = redo_count;
				p.rp_maxn = SG_REDO_REPLAY_MAX;
				st.launches++;
			} else if (nreg) {
				HIPCHK(launch_sorted(nreg, true, lgrid, lds, ts, p, redo_list, redo_count));
				st.launches++;
			} else {
				hipLaunchKernelGGL(k_redo_to_literal, dim3(64), dim3(256), 0, ts, p, (const unsigned int *)redo_list,
						(const unsigned int *)redo_count, 0xFFFFFFFFu);
				HIPCHK(hipGetLastError());
				st.launches++;
			}
		} else if (literal_all) {
			HIPCHK(hipEventRecord(cev[0], s));
			hipLaunchKernelGGL(k_list_all, dim3(1024), dim3(256), 0, s, p);
			HIPCHK(hipGetLastError());
			HIPCHK(hipEventRecord(cev[1], s));
			if (int rc = to_tail())
				return rc;
			st.launches = 1;
		} else {
			HIPCHK(hipEventRecord(cev[0], s));
			HIPCHK(launch_sorted(nreg, false, dim3((unsigned)nblk), lds, s, p, nullptr, nullptr));
			HIPCHK(hipEventRecord(cev[1], s));
			if (int rc = to_tail())
				return rc;
			st.main_kernel_blocks = (int)nblk;
			st.launches = 1;
		}
		/* exact wave-per-pixel replay of queued SIGMA / WINSORIZED pixels (the replay route's redo
		 * list, early breaks with this pixel's own stale rejected[]), then the literal path for what
		 * remains: two phases, grids read the count on the device */
		const unsigned lit_threads = lit_thread_count(N);
		HIPCHK(ensure(sb.scratch, lit_scratch_bytes(N)));
		if (d->method == SG_STACK_MEAN && (p.rejection == SG_SIGMA || p.rejection == SG_WINSORIZED) &&
				N <= SG_REPLAY_MAXN) {
			if (N <= 512)	/* the per-wave LDS sized for 512 frames (k_stack_replay<SG_REPLAY_FASTN>) */
				hipLaunchKernelGGL(k_stack_replay<512>, dim3(2048), dim3(64 * SG_REPLAY_WAVES), 0, ts, p);
			else
				hipLaunchKernelGGL(k_stack_replay<SG_REPLAY_MAXN>, dim3(2048), dim3(64 * SG_REPLAY_WAVES), 0, ts, p);
			HIPCHK(hipGetLastError());
			st.launches++;
		}
		for (int phase = 1; phase <= 2; phase++) {
			hipLaunchKernelGGL(k_stack_literal, dim3(lit_threads / 64), dim3(64), 0, ts, p, ct,
					0u, (uint8_t *)sb.scratch.p, phase);
			HIPCHK(hipGetLastError());
		}
		st.launches += 2;
	} else {
		if (int rc = flush_inputs())
			return rc;
		if (d->method == SG_STACK_SUM) {
			HIPCHK(ensure(dv.sum_buf, sizeof(uint32_t) * npix_img));
			p.sum_buf = (uint32_t *)dv.sum_buf.p;
		}
		dim3 grid((W + 255) / 256, nrows, C);
		/* pixel pairs per lane (dword loads) unless a plane is too large for a 31-bit offset */
		const bool pairs = W >= 2 && (uint64_t)W * (uint64_t)H * 2u < (1ull << 31) && ctx->knobs.reduce1 != 1;
		const dim3 grid2(((W + 1) / 2 + 255) / 256, nrows, C);
		/* XCD-aware SGPR-offset loads (k_stack_reduce3) when the shifted row offsets fit 32 bits,
		 * the per-lane pair kernel (SG_REDUCE1=2, A/B) otherwise */
		const bool r3 = pairs && hist_addr_ok && ctx->knobs.reduce1 == 0;
		/* 256-byte segments per wave: SEG = 1 by default (SG_REDUCE_SEG: 1 / 2 / 4, A/B; 2 and 4
		 * measured slower, profiles/r05g_reduce_seg_*) */
		const int seg = ctx->knobs.reduce_seg;
		const unsigned nb3 = (unsigned)(((W + 512 * seg - 1) / (512 * seg)) * (size_t)nrows * C);
		HIPCHK(hipEventRecord(cev[0], s));
		if (r3) {
			/* MEAN: the normalising instance's fp64 path costs registers: its own kernel */
			const int m = d->method == SG_STACK_SUM ? 0 : d->method == SG_STACK_MEAN ? (p.normalize ? 2 : 1) :
				d->method == SG_STACK_MAX ? 3 : 4;
			switch (m * 8 + seg) {
#define SG_R3L(M, G)                                                                            \
			case M * 8 + G:                                                                 \
				hipLaunchKernelGGL((k_stack_reduce3<M, G>), dim3(nb3), dim3(256), 0, s, p, p.hist_tab, p.shifty); \
				break;
			SG_R3L(0, 1) SG_R3L(0, 2) SG_R3L(0, 4)
			SG_R3L(1, 1) SG_R3L(1, 2) SG_R3L(1, 4)
			SG_R3L(2, 1) SG_R3L(2, 2) SG_R3L(2, 4)
			SG_R3L(3, 1) SG_R3L(3, 2) SG_R3L(3, 4)
			SG_R3L(4, 1) SG_R3L(4, 2) SG_R3L(4, 4)
#undef SG_R3L
			default:
				return set_err(ctx, SG_ERR_GENERIC, "no reduce kernel for this case%s%.0ld", "", 0);
			}
		} else if (pairs) {
			hipLaunchKernelGGL(k_stack_reduce2, grid2, dim3(256), 0, s, p);
		} else {
			hipLaunchKernelGGL(k_stack_reduce, grid, dim3(256), 0, s, p);
		}
		HIPCHK(hipGetLastError());
		HIPCHK(hipEventRecord(cev[1], s));
		st.main_kernel_blocks = r3 ? (int)nb3 : pairs ? (int)(grid2.x * grid2.y * grid2.z) : (int)(grid.x * grid.y * grid.z);
		st.launches = 1;
		if (d->method == SG_STACK_SUM && (sum_mode == SUM_WHOLE || sum_mode == SUM_LAST_BAND)) {
			/* the 65535/max scaling (:328-342) needs the maximum over the whole image: a
			 * streamed sequence finalises every row once its last band is summed */
			SgStackParams pf = p;
			dim3 gf = grid;
			if (sum_mode == SUM_LAST_BAND) {
				pf.row_begin = 0;
				pf.row_end = H;
				gf.y = H;
			}
			hipLaunchKernelGGL(k_sum_finalize, gf, dim3(256), 0, s, pf);
			HIPCHK(hipGetLastError());
			st.launches++;
		}
	}
	if (SG_DBG(p) == 12)
		sg_dbg_why_dump(ts);
	/* the counters back to the host: queued; a synchronous call folds them at once, an async one
	 * when its slot is needed again or at sg_stack_collect */
	hipLaunchKernelGGL(k_ctr_finalize, dim3(1), dim3(256), 0, ts, (unsigned long long *)cblk,
			dv.ctr_hd + (size_t)slot * (SG_CTR_HOSTB / sizeof(unsigned long long)));
	HIPCHK(hipGetLastError());
	dv.ctr_clean[slot] = true;
	HIPCHK(hipEventRecord(cev[2], ts));
	dv.pend_sum_read[slot] = d->method == SG_STACK_SUM;
	dv.pstats[slot] = st;
	dv.pend[slot] = true;
	dv.pend_seq[slot] = ++dv.seq;
	if (slot_out)
		*slot_out = slot;
	if (async)
		return SG_OK;
	return stack_fold(ctx, dv, slot, rej, maxim_out, true);
}

extern "C" int sg_stack_u16_device(sg_ctx *ctx, int dev_index, const sg_stack_desc *d,
		const uint16_t *d_frames, int64_t frame_stride, int64_t plane_stride, uint16_t *d_out,
		int row_begin, int row_end, uint64_t rej[3][2], uint64_t *maxim_out, void *stream) {
	const int rc = stack_device_core(ctx, dev_index, d, d_frames, frame_stride, plane_stride, d_out, row_begin,
			row_end, rej, maxim_out, stream, SUM_WHOLE);
	return rc == SG_ERR_WALK ? SG_ERR_GENERIC : rc;
}

/* the same call queued without waiting: its counters come back with sg_stack_collect */
extern "C" int sg_stack_u16_device_async(sg_ctx *ctx, int dev_index, const sg_stack_desc *d,
		const uint16_t *d_frames, int64_t frame_stride, int64_t plane_stride, uint16_t *d_out,
		int row_begin, int row_end, void *stream) {
	const int rc = stack_device_core(ctx, dev_index, d, d_frames, frame_stride, plane_stride, d_out, row_begin,
			row_end, nullptr, nullptr, stream, SUM_WHOLE, true);
	return rc == SG_ERR_WALK ? SG_ERR_GENERIC : rc;
}

/* `stream` waits (on the device, the host does not block) for every tail kernel queued so far by
 * SG_STACK_RESULT_AT_COLLECT calls of this device slot: they read d_frames and write d_out after
 * the call's own stream has moved on, so a caller that refills d_frames or reuses d_out on its
 * stream before sg_stack_collect orders the refill behind this */
extern "C" int sg_stack_wait_tail(sg_ctx *ctx, int dev_index, void *stream) {
	if (!ctx || dev_index < 0 || dev_index >= (int)ctx->dev.size())
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[(size_t)dev_index];
	if (!dv.tail)
		return SG_OK;
	HIPCHK(hipSetDevice(dv.id));
	HIPCHK(hipEventRecord(dv.tail_done_ev, dv.tail));
	HIPCHK(hipStreamWaitEvent(stream ? (hipStream_t)stream : dv.stream, dv.tail_done_ev, 0));
	return SG_OK;
}

extern "C" int sg_stack_collect(sg_ctx *ctx, int dev_index, uint64_t rej[3][2], uint64_t *maxim) {
	if (!ctx || dev_index < 0 || dev_index >= (int)ctx->dev.size())
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[(size_t)dev_index];
	HIPCHK(hipSetDevice(dv.id));
	while (dv.pend[0] || dv.pend[1]) {
		const int slot = (dv.pend[0] && (!dv.pend[1] || dv.pend_seq[0] < dv.pend_seq[1])) ? 0 : 1;
		stack_fold_acc(ctx, dv, slot);
	}
	const int rc = dv.acc_rc;
	if (rej)
		for (int c = 0; c < 3; c++) {
			rej[c][0] = dv.acc_rej[c][0];
			rej[c][1] = dv.acc_rej[c][1];
		}
	if (maxim)
		*maxim = dv.acc_max;
	for (int c = 0; c < 3; c++)
		dv.acc_rej[c][0] = dv.acc_rej[c][1] = 0;
	dv.acc_max = 0;
	dv.acc_rc = 0;
	return rc;
}

/* device bytes a stack call holds besides the frames: the output image (2 B per sample),
 * flag list and redo list (4 + 4 B), flag map (1 B), SUM's u32 sums (4 B), the literal
 * kernel's scratch, the readers' staging and the small tables */
static size_t fixed_device_bytes(int N, int W, int H, int C) {
	const size_t npix = (size_t)C * H * W;
	return npix * 15 + lit_scratch_bytes(N) + ((size_t)4 << 20) +
		(size_t)SG_PULL_READERS * 2 * SG_PULL_CHUNK_BYTES;
}

/* HBM the host-pull path may fill with frames on one device: SG_HOST_BUDGET_BYTES (tests: the
 * frame budget itself), else 85 % of the free device memory (plus what the context already holds
 * for frames) less the call's other buffers, split between the context slots that share the card */
static size_t host_budget(const sg_ctx *ctx, SgDevice &dv, int N, int W, int H, int C) {
	if (ctx->knobs.host_budget > 0)
		return (size_t)ctx->knobs.host_budget;
	size_t fr = 0, tot = 0;
	if (hipMemGetInfo(&fr, &tot) != hipSuccess)
		return 0;
	const size_t b = (size_t)((double)(fr + dv.frames.size + dv.out.size) * 0.85) / (size_t)std::max(1, dv.shared);
	const size_t fixed = fixed_device_bytes(N, W, H, C);
	return b > fixed ? b - fixed : 0;
}

/* state shared by the device threads and their readers of one sg_stack_u16 call */
struct PullCall {
	const sg_stack_desc *d;
	sg_read_region_fn pull;
	void *user;
	sg_should_continue_fn cont;
	void *cont_user;
	int sy_min, sy_max;
	bool multi;			/* more than one device: SUM scales after every device's band */
	std::mutex cont_mu;		/* the caller's get_thread_run is asked from one thread at a time */
	std::atomic<int> stop{0};	/* a reader failed or the caller cancelled: every thread winds down */
	bool keep_going() {
		if (stop.load())
			return false;
		if (!cont)
			return true;
		std::lock_guard<std::mutex> lk(cont_mu);
		if (stop.load())
			return false;
		if (!cont(cont_user)) {
			stop = 1;
			return false;
		}
		return true;
	}
};

static int ensure_readers(sg_ctx *ctx, SgDevice &dv, int nreaders, size_t elems) {
	if ((int)dv.readers.size() < nreaders)
		dv.readers.resize((size_t)nreaders);
	for (int r = 0; r < nreaders; r++) {
		SgReader &rd = dv.readers[(size_t)r];
		if (!rd.stream) {
			HIPCHK(hipStreamCreateWithFlags(&rd.stream, hipStreamNonBlocking));
			for (int k = 0; k < 2; k++)
				HIPCHK(hipEventCreateWithFlags(&rd.ev[k], hipEventDisableTiming));
		}
		if (rd.cap < elems) {
			for (int k = 0; k < 2; k++) {
				if (rd.used[k])
					HIPCHK(hipEventSynchronize(rd.ev[k]));
				rd.used[k] = false;
				if (rd.pin[k])
					(void)hipHostFree(rd.pin[k]);
				if (rd.dstage[k])
					(void)hipFree(rd.dstage[k]);
				rd.pin[k] = rd.dstage[k] = nullptr;
			}
			rd.cap = 0;
			for (int k = 0; k < 2; k++) {
				HIPCHK(hipHostMalloc((void **)&rd.pin[k], elems * sizeof(uint16_t)));
				HIPCHK(hipMalloc((void **)&rd.dstage[k], elems * sizeof(uint16_t)));
			}
			rd.cap = elems;
		}
	}
	return SG_OK;
}

/*
 * One band of frame rows onto one device: memory rows [lo, lo + nres) of every frame and
 * channel into `frames` (plane (i C + c) at (i C + c) nres W).  Like the reference's OpenMP
 * team reading its blocks (stacking.c:1513-1591, seq_opened_read_region under per-file locks),
 * `nreaders` host threads pull frames i = r, r + R, ... in top-down row chunks of at most
 * SG_PULL_CHUNK_BYTES into their two pinned buffers (the reader refills one while the other is
 * in flight), copy each chunk on their own stream and flip it into place on the device.  The
 * caller's cancellation is polled once per frame, as get_thread_run() is per frame read
 * (:1539).  Returns once every chunk has landed.
 */
static int pull_band(sg_ctx *ctx, SgDevice &dv, PullCall &pc, int nreaders, uint16_t *frames, int lo, int nres) {
	const sg_stack_desc *d = pc.d;
	const int N = d->nb_frames, W = d->width, H = d->height, C = d->nb_layers;
	const int chunk = (int)std::max<size_t>(1, SG_PULL_CHUNK_BYTES / ((size_t)W * sizeof(uint16_t)));
	const size_t bplane = (size_t)nres * W;
	std::atomic<int> rc{SG_OK};
	auto fail = [&](int code) {
		int expect = SG_OK;
		rc.compare_exchange_strong(expect, code);
		pc.stop = 1;
	};
	auto work = [&](int r) {
		SgReader &rd = dv.readers[(size_t)r];
		if (hipSetDevice(dv.id) != hipSuccess)
			return fail(set_err(ctx, SG_ERR_DEVICE, "hipSetDevice failed in a reader%s%ld", "", dv.id));
		int k = 0;
		for (int i = r; i < N; i += nreaders) {
			if (!pc.keep_going())
				return fail(SG_ERR_GENERIC);	/* cancelled, or another thread failed */
			for (int c = 0; c < C; c++) {
				uint16_t *plane = frames + ((size_t)i * C + c) * bplane;
				for (int m0 = 0; m0 < nres; m0 += chunk) {
					const int h = std::min(chunk, nres - m0);
					if (rd.used[k] && hipEventSynchronize(rd.ev[k]) != hipSuccess)
						return fail(set_err(ctx, SG_ERR_DEVICE, "staging event failed%s%ld", "", i));
					/* memory rows lo + m0 .. lo + m0 + h - 1 as the top-down area the
					 * region reader takes (y = H - 1 - the highest memory row) */
					const sg_rect area = {0, H - lo - m0 - h, W, h};
					if (pc.pull(pc.user, c, i, rd.pin[k], &area) < 0)
						return fail(set_err(ctx, SG_ERR_READ, "could not read frame%s %ld", "", i));
					if (hipMemcpyAsync(rd.dstage[k], rd.pin[k], (size_t)h * W * sizeof(uint16_t), hipMemcpyHostToDevice,
							rd.stream) != hipSuccess)
						return fail(set_err(ctx, SG_ERR_DEVICE, "upload failed for frame%s %ld", "", i));
					hipLaunchKernelGGL(k_flip_rows, dim3((unsigned)std::min(64, (W + 255) / 256), (unsigned)h), dim3(256), 0,
							rd.stream, (const uint16_t *)rd.dstage[k], plane + (size_t)m0 * W, W, h);
					if (hipGetLastError() != hipSuccess || hipEventRecord(rd.ev[k], rd.stream) != hipSuccess)
						return fail(set_err(ctx, SG_ERR_DEVICE, "flip launch failed for frame%s %ld", "", i));
					rd.used[k] = true;
					k ^= 1;
				}
			}
		}
	};
	std::vector<std::thread> th;
	int started = 1;
	for (int r = 1; r < nreaders; r++) {
		try {
			th.emplace_back(work, r);
			started++;
		} catch (...) {	/* no thread: the frames of the readers not started go unread -> fail */
			fail(set_err(ctx, SG_ERR_GENERIC, "could not start reader thread%s %ld", "", r));
			break;
		}
	}
	if (started == nreaders)
		work(0);
	for (std::thread &t : th)
		t.join();
	for (int r = 0; r < nreaders; r++)
		if (hipStreamSynchronize(dv.readers[(size_t)r].stream) != hipSuccess && rc.load() == SG_OK)
			fail(set_err(ctx, SG_ERR_DEVICE, "upload stream failed%s%ld", "", r));
	return rc.load();
}

/*
 * The rows [B, E) of the output on device g: banded under the device's HBM budget like the
 * reference's row blocks (stacking.c:1397-1476, sized from the memory budget :1903-1915); each
 * band's frame rows (the rows its shifts reach, :1544-1577) are pulled by the device's readers
 * and stacked with only those rows resident.  With two frame buffers (every method but SUM,
 * whose 65535/max scaling carries one maximum across the bands) band k + 1 is read while band k
 * stacks: the stack is queued without waiting (sg_stack_u16_device_async's path) and folded
 * once the next band has landed, as the reference's team reads blocks while other threads stack
 * theirs (:1513-1591).  The output rows stay in the device's dv.out (SUM of several devices:
 * raw sums, scaled once the maximum over every device is known).
 */
static int pull_device(sg_ctx *ctx, int g, PullCall &pc, int B, int E, int nreaders, uint64_t rej[3][2],
		uint64_t *maxim) {
	SgDevice &dv = ctx->dev[(size_t)g];
	const sg_stack_desc *d = pc.d;
	const int N = d->nb_frames, W = d->width, H = d->height, C = d->nb_layers;
	HIPCHK(hipSetDevice(dv.id));
	const int64_t halo = std::min<int64_t>((int64_t)pc.sy_max - pc.sy_min, H);
	const size_t row_bytes = (size_t)N * C * W * sizeof(uint16_t);	/* one row of every frame */
	const size_t budget = host_budget(ctx, dv, N, W, H, C);
	int band = E - B, nbuf = 1;
	if ((size_t)band * row_bytes > budget) {
		const int64_t fit = (int64_t)(budget / row_bytes) - halo;
		if (fit < 1)
			return set_err(ctx, SG_ERR_SIZE, "the sequence does not fit the device even one row at a "
					"time%s%.0ld", "", 0);
		band = (int)std::min<int64_t>(fit, band);
		/* several bands: two half-size buffers when a band of each still fits */
		const int64_t fit2 = (int64_t)(budget / 2 / row_bytes) - halo;
		if (d->method != SG_STACK_SUM && fit2 >= 1 && ctx->knobs.pull_overlap) {
			band = (int)std::min<int64_t>(fit2, band);
			nbuf = 2;
		}
	}
	const int64_t rows_cap = std::min<int64_t>(band + halo, H);
	const size_t buf_elems = (size_t)rows_cap * W * C * N;
	HIPCHK(ensure(dv.frames, nbuf * buf_elems * sizeof(uint16_t)));
	HIPCHK(ensure(dv.out, (size_t)W * H * C * sizeof(uint16_t)));
	const size_t chunk_elems = std::min<size_t>((size_t)rows_cap * W,
			std::max<size_t>(1, SG_PULL_CHUNK_BYTES / ((size_t)W * sizeof(uint16_t))) * W);
	if (int rc = ensure_readers(ctx, dv, nreaders, chunk_elems))
		return rc;
	for (int c = 0; c < 3; c++)
		rej[c][0] = rej[c][1] = 0;
	const bool banded = band < E - B || pc.multi;
	/* extra: rows above the band kept resident besides the halo.  A first-pass early break
	 * inherits the stale rejected[] of the previous pixel of the reference's OpenMP thread
	 * (stacking.c:1684), i.e. of the pixel one memory row up (rows run top-down inside a
	 * block); when that pixel lies above the band the core reports it (SG_ERR_WALK) and the
	 * band is retried narrower with more rows above it resident (same total rows) */
	int extra = 0;
	struct Pending {
		int slot, b, e, hi;
	} pend = {-1, 0, 0, 0};
	/* the band in flight: its counters, or a retry of it (the band start goes back to it) */
	auto fold = [&](int &b) -> int {
		uint64_t brej[3][2];
		const int rc = stack_fold(ctx, dv, pend.slot, brej, nullptr, true);
		const Pending pd = pend;
		pend.slot = -1;
		if (!pc.multi) {	/* one device: its folded band is the call's statistics (sg_get_last_stats) */
			std::lock_guard<std::mutex> lk(ctx->mu);
			ctx->stats = dv.stats;
		}
		if (rc == SG_ERR_WALK && pd.hi < H - 1 && pd.e - pd.b > 1) {
			extra = std::min(pd.e - pd.b - 1 + extra, extra ? 2 * extra : 4);
			b = pd.b;
			return 1;
		}
		if (rc)
			return rc == SG_ERR_WALK ? SG_ERR_GENERIC : rc;
		for (int c = 0; c < 3; c++) {
			rej[c][0] += brej[c][0];
			rej[c][1] += brej[c][1];
		}
		return SG_OK;
	};
	auto drain = [&]() {
		if (pend.slot >= 0) {
			(void)hipEventSynchronize(dv.cev[pend.slot][2]);
			dv.pend[pend.slot] = false;
			pend.slot = -1;
		}
	};
	int buf = 0;
	for (int b = B; b < E;) {
		const int e = std::min(E, b + std::max(1, band - extra));
		int lo = (int)std::max<int64_t>(0, (int64_t)b - pc.sy_max);
		int hi = (int)std::min<int64_t>(H - 1, (int64_t)e - 1 - pc.sy_min + extra);
		if (lo > hi)	/* every row of the band is shifted out of the frames: nothing is read */
			lo = hi = std::min(b, H - 1);
		const int nres = hi - lo + 1;
		const size_t bplane = (size_t)nres * W;
		uint16_t *fb = (uint16_t *)dv.frames.p + (size_t)buf * buf_elems;
		if (int rc = pull_band(ctx, dv, pc, nreaders, fb, lo, nres)) {
			drain();
			return rc;
		}
		if (pend.slot >= 0) {	/* the previous band stacked while this one was read */
			int bb = b;
			const int rc = fold(bb);
			if (rc < 0)
				return rc;
			if (rc == 1) {	/* retry it narrower: this band's rows are read again afterwards */
				b = bb;
				continue;
			}
		}
		sg_stack_desc bd = *d;
		bd.resident_rows[0] = lo;
		bd.resident_rows[1] = hi + 1;
		const int sum_mode = d->method != SG_STACK_SUM || !banded ? SUM_WHOLE
			: b == B ? SUM_FIRST_BAND : (!pc.multi && e == H) ? SUM_LAST_BAND : SUM_MID_BAND;
		/* base pointer biased so that memory row r of a frame plane sits at r*W */
		const uint16_t *base = fb - (ptrdiff_t)lo * W;
		if (nbuf == 2) {
			int slot = -1;
			if (int rc = stack_device_core(ctx, g, &bd, base, (int64_t)bplane * C, (int64_t)bplane,
					(uint16_t *)dv.out.p, b, e, nullptr, nullptr, dv.stream, sum_mode, true, &slot)) {
				drain();
				return rc == SG_ERR_WALK ? SG_ERR_GENERIC : rc;
			}
			pend = {slot, b, e, hi};
			buf ^= 1;
			b = e;
			if (b >= E) {	/* the last band: fold it here (a retry loops back) */
				const int rc = fold(b);
				if (rc < 0)
					return rc;
			}
			continue;
		}
		uint64_t brej[3][2];
		int rc = stack_device_core(ctx, g, &bd, base, (int64_t)bplane * C, (int64_t)bplane, (uint16_t *)dv.out.p, b,
				e, brej, maxim, dv.stream, sum_mode);
		if (rc == SG_ERR_WALK && hi < H - 1 && band - extra > 1) {
			extra = std::min(band - 1, extra ? 2 * extra : 4);
			continue;	/* same band start, narrower band, more rows above resident */
		}
		if (rc)
			return rc == SG_ERR_WALK ? SG_ERR_GENERIC : rc;
		for (int c = 0; c < 3; c++) {
			rej[c][0] += brej[c][0];
			rej[c][1] += brej[c][1];
		}
		b = e;
	}
	return SG_OK;
}

/* SUM over several devices: the 65535/max scaling of stack_summing (:328-342) with the maximum
 * over the whole image, applied to device g's rows [B, E) of raw sums */
static int sum_finalize_rows(sg_ctx *ctx, int g, int W, int H, int C, int B, int E, unsigned int gmax) {
	SgDevice &dv = ctx->dev[(size_t)g];
	HIPCHK(hipSetDevice(dv.id));
	SgStackParams p;
	memset(&p, 0, sizeof p);
	p.W = W;
	p.H = H;
	p.C = C;
	p.out = (uint16_t *)dv.out.p;
	p.sum_buf = (uint32_t *)dv.sum_buf.p;
	p.row_begin = B;
	p.row_end = E;
	p.maxim = (unsigned int *)((char *)dv.ctr.p + SG_CTR_REJB + 64);
	HIPCHK(hipMemcpyAsync(p.maxim, &gmax, sizeof gmax, hipMemcpyHostToDevice, dv.stream));
	hipLaunchKernelGGL(k_sum_finalize, dim3((unsigned)((W + 255) / 256), (unsigned)(E - B), (unsigned)C), dim3(256), 0,
			dv.stream, p);
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(dv.stream));
	return SG_OK;
}

/*
 * host-pull path: frames come through seq_opened_read_region-shaped callbacks.  Every device of
 * the context takes a contiguous share of the output rows (the reference's row blocks are the
 * natural shard) and is driven by its own host thread, whose readers pull and upload
 * that share's frame rows directly (no device relays another's data); each device's band is
 * copied back into `out`, the rejection counters are summed.
 */
extern "C" int sg_stack_u16(sg_ctx *ctx, const sg_stack_desc *d, sg_read_region_fn pull, void *user,
		sg_should_continue_fn cont, void *cont_user, uint16_t *out, uint64_t rej[3][2],
		uint64_t *maxim) {
	if (!ctx || !d || !pull || !out || ctx->dev.empty())
		return SG_ERR_GENERIC;
	const int N = d->nb_frames, W = d->width, H = d->height, C = d->nb_layers;
	if (N < 2)
		return set_err(ctx, SG_ERR_GENERIC, "select at least two frames%s (%ld)", "", N);
	if (W <= 0 || H <= 0 || C < 1 || C > 3)
		return SG_ERR_SIZE;
	PullCall pc;
	pc.d = d;
	pc.pull = pull;
	pc.user = user;
	pc.cont = cont;
	pc.cont_user = cont_user;
	/* frame rows a band reads: [b - sy_max, e - 1 - sy_min] */
	const bool use_shift = d->method != SG_STACK_MEDIAN && d->shiftx && d->shifty;
	pc.sy_min = pc.sy_max = 0;
	for (int i = 0; use_shift && i < N; i++) {
		pc.sy_min = i ? std::min(pc.sy_min, d->shifty[i]) : d->shifty[i];
		pc.sy_max = i ? std::max(pc.sy_max, d->shifty[i]) : d->shifty[i];
	}
	const int G = (int)std::min<size_t>(ctx->dev.size(), (size_t)H);
	pc.multi = G > 1;
	/* readers per device: the reference's team size (com.max_thread) shared between the
	 * devices, at least one, at most SG_PULL_READERS */
	const int team = d->max_thread > 0 ? d->max_thread : default_threads();
	const int nreaders = std::max(1, std::min(SG_PULL_READERS, team / G));
	std::vector<int> rb((size_t)G + 1);
	for (int g = 0; g <= G; g++)
		rb[(size_t)g] = (int)((int64_t)g * H / G);
	std::vector<int> rcs((size_t)G, SG_OK);
	std::vector<std::array<uint64_t, 6>> rj((size_t)G);
	std::vector<uint64_t> mx((size_t)G, 0);
	/* SUM over several devices scales with the maximum over all of them (after the join);
	 * every other result leaves its device from the device's own thread */
	const bool late_copy = d->method == SG_STACK_SUM && pc.multi;
	auto copy_out = [&](int g) -> int {
		SgDevice &dv = ctx->dev[(size_t)g];
		const int B = rb[(size_t)g], E = rb[(size_t)g + 1];
		HIPCHK(hipSetDevice(dv.id));
		for (int c = 0; c < C; c++) {
			const size_t o = ((size_t)c * H + B) * W;
			HIPCHK(hipMemcpy(out + o, (const uint16_t *)dv.out.p + o, (size_t)(E - B) * W * sizeof(uint16_t),
					hipMemcpyDeviceToHost));
		}
		return SG_OK;
	};
	auto run = [&](int g) {
		uint64_t r6[3][2];
		int r = pull_device(ctx, g, pc, rb[(size_t)g], rb[(size_t)g + 1], nreaders, r6, &mx[(size_t)g]);
		if (r == SG_OK && !late_copy)
			r = copy_out(g);
		rcs[(size_t)g] = r;
		if (r)
			pc.stop = 1;
		memcpy(rj[(size_t)g].data(), r6, sizeof r6);
	};
	{
		std::vector<std::thread> th;
		bool started = true;
		for (int g = 1; g < G; g++) {
			try {
				th.emplace_back(run, g);
			} catch (...) {
				rcs[(size_t)g] = set_err(ctx, SG_ERR_GENERIC, "could not start the thread of device slot%s %ld", "", g);
				pc.stop = 1;
				started = false;
				break;
			}
		}
		if (started)
			run(0);
		else
			rcs[0] = SG_ERR_GENERIC;
		for (std::thread &t : th)
			t.join();
	}
	/* a device's own failure wins over the stop (SG_ERR_GENERIC) it caused in the others;
	 * a cancellation alone is SG_ERR_GENERIC, as get_thread_run() going false is (-1) */
	int rc = SG_OK;
	for (int g = 0; g < G && rc == SG_OK; g++)
		if (rcs[(size_t)g] != SG_ERR_GENERIC)
			rc = rcs[(size_t)g];
	for (int g = 0; g < G && rc == SG_OK; g++)
		rc = rcs[(size_t)g];
	if (rc) {
		for (int g = 0; g < G; g++) {
			(void)hipSetDevice(ctx->dev[(size_t)g].id);
			(void)hipStreamSynchronize(ctx->dev[(size_t)g].stream);
		}
		return rc;
	}
	uint64_t gmax = 0;
	for (int g = 0; g < G; g++)
		gmax = std::max(gmax, mx[(size_t)g]);
	for (int g = 0; g < G && late_copy; g++) {
		if (int r = sum_finalize_rows(ctx, g, W, H, C, rb[(size_t)g], rb[(size_t)g + 1], (unsigned int)gmax))
			return r;
		if (int r = copy_out(g))
			return r;
	}
	if (rej)
		for (int c = 0; c < 3; c++) {
			rej[c][0] = rej[c][1] = 0;
			for (int g = 0; g < G; g++) {
				rej[c][0] += rj[(size_t)g][(size_t)c * 2];
				rej[c][1] += rj[(size_t)g][(size_t)c * 2 + 1];
			}
		}
	if (maxim)
		*maxim = gmax;
	if (pc.multi) {	/* the call's statistics over every device */
		sg_stack_stats agg;
		memset(&agg, 0, sizeof agg);
		for (int g = 0; g < G; g++) {
			const sg_stack_stats &s = ctx->dev[(size_t)g].stats;
			agg.kernel_ms = std::max(agg.kernel_ms, s.kernel_ms);
			agg.total_ms = std::max(agg.total_ms, s.total_ms);
			agg.slow_pixels += s.slow_pixels;
			agg.chain_pixels += s.chain_pixels;
			agg.compact_pixels += s.compact_pixels;
			agg.exported_pixels += s.exported_pixels;
			agg.norm_fma = std::max(agg.norm_fma, s.norm_fma);
			agg.launches += s.launches;
			agg.main_kernel_blocks += s.main_kernel_blocks;
			agg.path = s.path;
		}
		std::lock_guard<std::mutex> lk(ctx->mu);
		ctx->stats = agg;
	}
	return SG_OK;
}

extern "C" int sg_synth_fill_frames_device(sg_ctx *ctx, int dev_index, uint16_t *d_frames, int first_frame,
		int nframes, int nb_layers, int height, int width, int row_begin, int row_end, uint64_t seed,
		int maxshift, int64_t frame_stride, int64_t plane_stride, void *stream) {
	if (!ctx || dev_index < 0 || dev_index >= (int)ctx->dev.size() || first_frame < 0)
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[dev_index];
	HIPCHK(hipSetDevice(dv.id));
	hipStream_t s = stream ? (hipStream_t)stream : dv.stream;
	hipLaunchKernelGGL(k_synth_fill, dim3(8192), dim3(256), 0, s, d_frames, first_frame, nframes, nb_layers,
			height, width, row_begin, row_end, seed, maxshift,
			frame_stride > 0 ? frame_stride : (int64_t)nb_layers * height * width,
			plane_stride > 0 ? plane_stride : (int64_t)height * width);
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(s));
	return SG_OK;
}

extern "C" int sg_synth_fill_device(sg_ctx *ctx, int dev_index, uint16_t *d_frames, int nframes,
		int nb_layers, int height, int width, int row_begin, int row_end, uint64_t seed,
		int maxshift, int64_t frame_stride, void *stream) {
	return sg_synth_fill_frames_device(ctx, dev_index, d_frames, 0, nframes, nb_layers, height, width, row_begin,
			row_end, seed, maxshift, frame_stride, 0, stream);
}

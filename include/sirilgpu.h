/*
 * sirilgpu.h - C ABI of libsirilgpu.so, the MI355X (gfx950) implementation of Siril 0.9's
 * sequence registration + stacking hot path.
 *
 * Plain C types only (no torch, no HIP types in signatures).  Each entry point cites the
 * reference interface whose body it replaces; the reference-side glue is shown in
 * INTEGRATION.md.
 *
 * Conventions:
 *   - WORD = uint16_t (src/core/siril.h:44).
 *   - Images are planar per channel and bottom-up ("memory order", src/core/siril.h:391-442).
 *   - A region read through sg_read_region_fn is a top-down band, exactly what
 *     seq_opened_read_region() returns (src/io/sequence.c:690-700).
 *   - Return codes mirror the reference: 0 ok, -1 generic/cancel/unsupported, -2 size or
 *     allocation error, -3 read failure (src/stacking/stacking.c:244-246,1212-1220).
 *   - Device work runs on the context's own non-blocking HIP stream (or the stream passed
 *     in): device buffers handed to a *_device call must be complete, i.e. the caller
 *     synchronises whatever produced them on other streams (a torch fill, a copy) first.
 */
#ifndef SIRILGPU_H
#define SIRILGPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_OK 0
#define SG_ERR_GENERIC -1
#define SG_ERR_SIZE -2
#define SG_ERR_READ -3
#define SG_ERR_DEVICE -10

/* stacking_methods[] order, src/stacking/stacking.c:54-56 */
enum sg_stack_method {
	SG_STACK_SUM = 0,	/* stack_summing            :196-355  */
	SG_STACK_MEAN = 1,	/* stack_mean_with_rejection :1189-1858 */
	SG_STACK_MEDIAN = 2,	/* stack_median             :362-816  */
	SG_STACK_MAX = 3,	/* stack_addmax             :824-972  */
	SG_STACK_MIN = 4	/* stack_addmin             :979-1128 */
};

/* src/stacking/stacking.h:14-21 */
enum sg_rejection { SG_NO_REJEC, SG_PERCENTILE, SG_SIGMA, SG_SIGMEDIAN, SG_WINSORIZED, SG_LINEARFIT };
/* src/stacking/stacking.h:24-30 */
enum sg_normalization { SG_NO_NORM, SG_ADDITIVE, SG_MULTIPLICATIVE, SG_ADDITIVE_SCALING,
	SG_MULTIPLICATIVE_SCALING };

/* kernel selection for sg_stack_desc.kernel_path (results are identical on every path) */
enum sg_kernel_path { SG_PATH_AUTO = 0, SG_PATH_SORTED = 1 };

/* rectangle, src/core/siril.h:477-479 */
typedef struct { int x, y, w, h; } sg_rect;

/* shape of seq_opened_read_region (src/io/sequence.h:17): fill `buffer` with the top-down
 * band `area` of channel `layer` of frame `index`; <0 on failure */
typedef int (*sg_read_region_fn)(void *user, int layer, int index, uint16_t *buffer,
		const sg_rect *area);
/* get_thread_run() (src/core/processing.c:294-300): 0 = cancel requested */
typedef int (*sg_should_continue_fn)(void *user);

/* What a stack_method needs from struct stacking_args + sequence (src/stacking/stacking.h:38-56,
 * src/core/siril.h:328-374), flattened to plain arrays.  Per-frame arrays are indexed by the
 * stacked-frame position i (the reference's image_indices[i] order). */
typedef struct {
	int method;		/* enum sg_stack_method */
	int rejection;		/* enum sg_rejection (SG_STACK_MEAN only) */
	int normalize;		/* enum sg_normalization (MEAN and MEDIAN) */
	double sig[2];		/* args->sig */
	int nb_frames;		/* args->nb_images_to_stack */
	int width, height, nb_layers;	/* seq->rx, seq->ry, naxes[2] */
	const int *shiftx;	/* regparam[reglayer][image_indices[i]].shiftx, or NULL */
	const int *shifty;	/* ... .shifty, or NULL (no registration data) */
	const double *offset;	/* normalisation coefficients (compute_normalization), or NULL */
	const double *mul;
	const double *scale;
	int max_thread;		/* com.max_thread: the reference's OpenMP team size */
	int max_number_of_rows;	/* args->max_number_of_rows */
	int kernel_path;	/* SG_PATH_*: 0 = automatic (no reference equivalent; testing/A-B) */
	/* memory rows [resident_rows[0], resident_rows[1]) of every frame are present at
	 * d_frames (sg_stack_u16_device); {0, 0} = all rows [0, height).  No reference
	 * equivalent: it lets a rank hold only its row band plus the rows its shifts reach. */
	int resident_rows[2];
	int flags;		/* SG_STACK_* flags below (0 = none) */
	int reserved[2];
} sg_stack_desc;
/* sg_stack_desc.flags: the output is needed only once sg_stack_collect has returned, so an
 * async call (sg_stack_u16_device_async) may run its work after the main kernel (redo lists,
 * replay, counters) beside the next call's main kernel instead of on `stream`.  That work still
 * READS d_frames and WRITES d_out after `stream` has moved on: both must stay unchanged (the
 * frames) and unread (the output) until sg_stack_collect returns, or until work queued on a
 * stream after sg_stack_wait_tail(ctx, dev, stream) */
#define SG_STACK_RESULT_AT_COLLECT 1

typedef struct sg_ctx sg_ctx;

/* Open the devices this context drives: devs[0..ndev) (NULL: 0..ndev-1), ndev = 0 device 0,
 * ndev < 0 every visible device.  An id may repeat (context slots sharing one card).  One HIP
 * stream per slot; the host-pull calls (sg_stack_u16, sg_register_dft_u16) drive every slot
 * from its own host thread. */
int sg_init(sg_ctx **ctx, int ndev, const int *devs);
void sg_shutdown(sg_ctx *ctx);
const char *sg_last_error(const sg_ctx *ctx);

/*
 * Host-pull stack: replaces the bodies of stack_summing / stack_mean_with_rejection /
 * stack_median / stack_addmax / stack_addmin (src/stacking/stacking.c:196,1189,362,824,979).
 * Every device of the context takes a contiguous share of the output rows (the reference's
 * row blocks, :1397-1476, are the natural shard) and is driven by its own host thread, whose
 * readers (the reference's team size max_thread shared between the devices, at most 8 per
 * device) pull that share's frame rows through `pull` (seq_opened_read_region shape, called
 * concurrently as the reference's OpenMP team does) into pinned staging and upload them
 * directly to that device; a share larger than the device's HBM budget is stacked in row bands.
 * The result is written bottom-up into `out` (nb_layers*H*W WORDs, the buffer the reference
 * hands to gfit.data).  rej receives the per-channel low/high rejection counters of
 * :1796-1817 (MEAN only, summed over the devices), maxim the sum maximum of :311-313 (SUM only,
 * over the whole image; the 65535/max scaling uses it on every device).  `cont` is polled once
 * per frame read (get_thread_run, :1539); a cancellation returns SG_ERR_GENERIC.
 */
int sg_stack_u16(sg_ctx *ctx, const sg_stack_desc *desc, sg_read_region_fn pull, void *user,
		sg_should_continue_fn cont, void *cont_user, uint16_t *out, uint64_t rej[3][2],
		uint64_t *maxim);

/*
 * Device-resident stack (frames already in HBM).  d_frames holds frame i, channel c, memory
 * row r, column x at d_frames[i*frame_stride + c*plane_stride + r*width + x].  Output rows
 * [row_begin, row_end) (memory order) of every channel are written to d_out (same indexing
 * as a [C][H][W] image).  `stream` is a hipStream_t (NULL = the context's stream of device
 * `dev_index`).  The call is synchronous.
 *
 * Row bands (one rank per band): the band's output rows read frame rows
 * [row_begin - max(shifty), row_end - min(shifty)) (clipped to the frame), and those rows
 * must lie inside desc->resident_rows (else SG_ERR_SIZE); a rank holding only them may pass a
 * base pointer biased by -resident_rows[0]*width.  A rejection stack whose FIRST sigma pass
 * breaks early (`N - r <= 4`, stacking.c:1684) reads the previous pixel's stale rejected[]
 * (SURVEY §8a a3 iii); the previous pixel in the reference's OpenMP thread order can lie
 * outside the band, and is then recomputed from the frames.  If its rows are not resident
 * the call fails with SG_ERR_GENERIC instead of guessing: for such stacks (in practice
 * small N with strong rejection) make the full frames resident.
 *
 * Refused regime (both entry points): a MEAN stack (stack_mean_with_rejection, any rejection;
 * stack_median ignores shifts) whose shifts make a row block
 * of the reference's partition (max_thread, max_number_of_rows; :1397-1476) with start_row > 0
 * read above the frame.  The reference then writes offset = W*(area.y - shifty) past its block
 * buffer (stacking.c:1555-1561, a heap overflow with an undefined result); the call fails with
 * SG_ERR_GENERIC and a message instead of zero-filling.  Keep |shifty| below the block height.
 * Second refused regime: a SIGMEDIAN pixel whose clipping loop (stacking.c:1696-1709, no pass
 * cap) never ends, i.e. a pass replaces samples by the values they already hold (e.g. {0, 0,
 * 1, 1} with sig[1] < 0.87) or the pixel needs more than 4096 passes; Siril hangs there, the
 * call fails with SG_ERR_GENERIC.
 */
int sg_stack_u16_device(sg_ctx *ctx, int dev_index, const sg_stack_desc *desc,
		const uint16_t *d_frames, int64_t frame_stride, int64_t plane_stride,
		uint16_t *d_out, int row_begin, int row_end, uint64_t rej[3][2], uint64_t *maxim,
		void *stream);
/*
 * The same stack queued without waiting for it (replaces the same loop body as
 * sg_stack_u16_device, for callers that keep several stacks in flight, e.g. a row band per call
 * in a loop: the host prepares the next call while the device works).  Every launch decision is
 * made on the device, so nothing here waits for the GPU except reusing a counter slot: at most
 * two calls per device slot are pending, a third folds the oldest.  Successive async calls of a
 * device slot must use one stream.  sg_stack_collect waits for every pending call of the slot
 * and returns the SUM of their rejection counters, the maximum of their SUM maxima and the first
 * error any of them met (SG_ERR_GENERIC for the refused regimes above); statistics then describe
 * the last folded call.
 */
int sg_stack_u16_device_async(sg_ctx *ctx, int dev_index, const sg_stack_desc *desc,
		const uint16_t *d_frames, int64_t frame_stride, int64_t plane_stride,
		uint16_t *d_out, int row_begin, int row_end, void *stream);
int sg_stack_collect(sg_ctx *ctx, int dev_index, uint64_t rej[3][2], uint64_t *maxim);
/* device-side ordering for SG_STACK_RESULT_AT_COLLECT calls (no reference equivalent: the
 * reference's blocks are synchronous): work queued on `stream` (NULL = the slot's own stream)
 * after this returns waits for every tail kernel the slot's async calls have queued so far, so
 * a band loop may refill d_frames, or read / send d_out, on its stream without a host wait */
int sg_stack_wait_tail(sg_ctx *ctx, int dev_index, void *stream);

/* Statistics of the last stack call on this context (for bench.py / rocprof cross-checks). */
typedef struct {
	double kernel_ms;	/* HIP-event time of the main stacking kernel(s) on their stream */
	double total_ms;	/* HIP-event time of the whole device-side stack call */
	uint64_t slow_pixels;	/* pixels re-done by the literal (fp80) path */
	uint64_t chain_pixels;	/* pixels needing the cross-pixel stale-state replay */
	uint64_t launches;	/* kernels launched by the main path */
	int main_kernel_blocks;
	int path;		/* main path of a MEAN stack: 1 = histogram (k_stack_hist), 0 = other */
	/* last registration: frames whose correlation maximum was a near tie, decided by exact
	 * integer correlations / left to the FFT arg-max (more candidates than the cap) */
	uint64_t reg_ties_resolved, reg_ties_unresolved;
	uint64_t reg_fp64_reruns;	/* pairs of the fp32 passes re-run in fp64 (near ties at fp32 tolerance) */
	uint64_t compact_pixels;	/* normalised histogram stacks: redo pixels whose sorted columns the
					 * histogram kernel wrote out (no gather in the sorted kernel) */
	double reg_ms;			/* last registration on a device: HIP-event span of its device work
					 * (first pass to the quality estimate's end, host waits included) */
	uint64_t exported_pixels;	/* histogram WINSORIZED: columns finished by k_hist_slow (SG_WINS_EXPORT) */
	int64_t norm_fma;		/* normalised histogram stack: the sample load found equal to the reference's roundings
					 * for every u16 value of every frame: 2 = an integer offset (additive, scale 1), 1 = one
					 * fma per sample; 0 = the reference's operations */
} sg_stack_stats;
int sg_get_last_stats(const sg_ctx *ctx, sg_stack_stats *st);
/* device slots of the context (sg_init's ndev): callers size their batches by it, as the
 * reference sizes its work by com.max_thread (src/core/siril.h:596) */
int sg_device_count(const sg_ctx *ctx, int *ndev);

/*
 * Per-frame normalisation statistics: location / scale of layer 0 as
 * statistics(fit, 0, NULL, STATS_IKSS, STATS_ZERO_NULLCHECK) computes them
 * (src/algos/statistics.c:152-326; the imstats _compute_normalization_for_image reads,
 * src/stacking/stacking.c:79-123).  d_frames: nframes frames [C][H][W] in Siril memory order
 * at frame_stride elements (0 = C*H*W); location / scale: host arrays [nframes].
 * 0, or SG_ERR_GENERIC when a frame has no non-zero pixel (statistics() returns NULL).
 */
int sg_frame_stats_ikss_device(sg_ctx *ctx, int dev_index, const uint16_t *d_frames, int nframes, int C,
		int H, int W, int64_t frame_stride, double *location, double *scale, void *stream);
/* the same on host frames (what seq_get_imstats computes from a loaded frame) */
int sg_frame_stats_ikss(sg_ctx *ctx, const uint16_t *frames, int nframes, int C, int H, int W,
		double *location, double *scale);
/* compute_normalization (src/stacking/stacking.c:125-190): offset / mul / scale [nframes]
 * from per-frame location / scale (host arithmetic; ref_image -1 = 0) */
int sg_compute_normalization(int mode, int nframes, int ref_image, const double *location,
		const double *scale_in, double *offset, double *mul, double *scale);

/*
 * DFT registration: replaces register_shift_dft (src/registration/registration.c:182-400).
 * d_sel / sel hold nframes bottom-up S x S selections (what seq_read_frame_part returns,
 * src/io/sequence.c:567-609), any side 4 <= S <= 4096 (FFTW plans every size, :251-257).
 * included may be NULL (process_all_frames).  Outputs the integer shifts and the normalised
 * quality (normalizeQualityData :163-176) per frame.  A correlation maximum whose runner-up
 * lies within the FFT tolerance is decided by exact integer correlations (sg_stack_stats
 * reg_ties_*).
 */
int sg_register_dft_u16(sg_ctx *ctx, const uint16_t *sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality);
/* the same with the qualities left RAW (QualityEstimate of the reference and of every
 * registered frame): the glue replays the reference's q_min / q_max / q_index bookkeeping and
 * normalizeQualityData itself, which a cancelled registration skips (registration.c:166-168).
 * Host selections: with several devices in the context the frames are split into contiguous
 * shards, one host thread per device. */
int sg_register_dft_u16_raw(sg_ctx *ctx, const uint16_t *sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality_raw);
int sg_register_dft_u16_device(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes,
		int S, int ref_image, const int *included, int *shiftx, int *shifty,
		double *quality, void *stream);
/*
 * The same on a shard of the sequence's frames (frame sharding over GPUs):
 * quality is left RAW (QualityEstimate per registered frame and the reference,
 * src/algos/quality.c:46-218; NaN where no pixel passes the threshold), so the caller can
 * gather every shard's values and apply normalizeQualityData (registration.c:163-176) with
 * the reference's min/max loop over all frames (sirilgpu_dist.register_sharded).  Frames
 * outside `included` are neither registered nor written.
 */
int sg_register_dft_u16_device_raw(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes,
		int S, int ref_image, const int *included, int *shiftx, int *shifty,
		double *quality_raw, void *stream);

/*
 * The same on selections read IN PLACE from resident frames (no extraction copy): selection f,
 * bottom-up row r, column x at d_sel[f * frame_pitch + r * row_pitch + x] (elements; row_pitch >=
 * S), e.g. a window of layer `layer` of [C][H][W] frames: d_sel = frames + layer H W + y0 W + x0,
 * frame_pitch = C H W, row_pitch = W.  What seq_read_frame_part (src/io/sequence.c:567-609)
 * extracts per frame is thus read by the first pass itself.  raw_quality != 0: the quality is
 * left raw as in sg_register_dft_u16_device_raw.
 */
int sg_register_dft_u16_device_pitched(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int64_t frame_pitch,
		int64_t row_pitch, int nframes, int S, int ref_image, const int *included, int *shiftx, int *shifty,
		double *quality, int raw_quality, void *stream);

/*
 * Perspective warp: replaces cvTransformImage (src/opencv/opencv.cpp:242-309) as the
 * star-alignment registration uses it (src/registration/registration.c:719-723, flip /
 * warp / flip): memory-order (bottom-up) planes in, memory-order planes out of size
 * out_width x out_height (ref.x, ref.y); hom = Homography h00..h22 row-major (the
 * forward map, inverted as warpPerspective does without WARP_INVERSE_MAP);
 * interpolation = opencv_interpolation (src/core/siril.h:257-264: 0 nearest, 1 linear,
 * 2 area (= linear), 3 cubic, 4 lanczos4), border constant 0.  OpenCV's algorithm is
 * restated (sg_warp.hip); OpenCV is unpinned, so parity is unpinned.
 */
int sg_warp_u16(sg_ctx *ctx, const uint16_t *in, int width, int height, int nb_layers,
		uint16_t *out, int out_width, int out_height, const double *hom, int interpolation);
int sg_warp_u16_device(sg_ctx *ctx, int dev_index, const uint16_t *d_in, int width, int height,
		int nb_layers, uint16_t *d_out, int out_width, int out_height, const double *hom,
		int interpolation, void *stream);

/* Synthetic sequence generator of include/sg_synth.h on the device (bench / tests):
 * frame f, channel c, row r at d_frames[f*frame_stride + (c*height + r)*width]
 * (frame_stride 0 = nb_layers*height*width). */
int sg_synth_fill_device(sg_ctx *ctx, int dev_index, uint16_t *d_frames, int nframes,
		int nb_layers, int height, int width, int row_begin, int row_end, uint64_t seed,
		int maxshift, int64_t frame_stride, void *stream);
/* the same for frames [first_frame, first_frame + nframes) of the sequence, written from d_frames
 * (a rank's block of a frame-sharded sequence), channel c at c * plane_stride (0 = height *
 * width): row r of channel c of local frame f at d_frames[f*frame_stride + c*plane_stride + r*width]
 * (a band-resident layout passes a base pointer biased by -row_begin*width) */
int sg_synth_fill_frames_device(sg_ctx *ctx, int dev_index, uint16_t *d_frames, int first_frame,
		int nframes, int nb_layers, int height, int width, int row_begin, int row_end, uint64_t seed,
		int maxshift, int64_t frame_stride, int64_t plane_stride, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SIRILGPU_H */

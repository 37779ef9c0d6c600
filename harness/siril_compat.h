/*
 * siril_compat.h - GTK-free restatement of the Siril 0.9 data model the stackers and the DFT
 * registration receive, with the reference's field order and types (so the glue in
 * siril_glue.c compiles unchanged inside Siril, where the real headers replace this one):
 *
 *   struct image_stats / imstats      src/core/siril.h:600-605
 *   struct imdata / imgdata           src/core/siril.h:293-303
 *   struct registration_data/regdata  src/core/siril.h:316-326
 *   struct sequ / sequence            src/core/siril.h:328-374
 *   struct ffit / fits                src/core/siril.h:391-442
 *   rectangle                         src/core/siril.h:477-479
 *   struct stacking_args (+ enums)    src/stacking/stacking.h:14-56
 *   struct registration_args          src/registration/registration.h:12-32
 *   seq_image_filter                  src/core/processing.h:5
 *
 * GLib types are spelled out (gboolean = int, gchar = char).  Types the hot path never
 * dereferences (layer_info, fitted_PSF, struct ser_struct, fitsfile) stay incomplete.
 * Configure-dependent members follow the reference build this restates: OpenMP on (the
 * fd_lock pointer exists, as an opaque pointer), FFMS2 off (no SEQ_AVI / film_file / ext).
 */
#ifndef SIRIL_COMPAT_H
#define SIRIL_COMPAT_H

#include <stdint.h>
#include <sys/time.h>

typedef unsigned short WORD;	/* src/core/siril.h:44 */
typedef int gboolean;
typedef char gchar;
#ifndef TRUE
#define TRUE 1
#define FALSE 0
#endif

#define USHORT_IMG 20	/* cfitsio bitpix codes */
#define TSTRING 16	/* cfitsio datatype codes */
#define TDOUBLE 82
#define BYTE_IMG 8
#define FLEN_VALUE 71	/* cfitsio fitsio.h */
#define PREVIEW_NB 2	/* src/core/siril.h:171 */
#define MAX_SEQPSF 7	/* src/core/siril.h:48 */
#define RLAYER 0
#define GLAYER 1
#define BLAYER 2

typedef struct fitsfile fitsfile;
typedef struct layer_info_struct layer_info;
typedef struct fwhm_struct fitted_PSF;
struct ser_struct;

typedef struct image_stats {
	long total, ngoodpix;
	double mean, avgDev, median, sigma, bgnoise, min, max, normValue, mad, sqrtbwmv,
			location, scale;
	char layername[6];
} imstats;

typedef struct imdata {
	int filenum;
	gboolean incl;
	imstats *stats;
	char *date_obs;
} imgdata;

typedef struct registration_data {
	int shiftx, shifty;
	float rot_centre_x, rot_centre_y;
	float angle;
	fitted_PSF *fwhm_data;
	float fwhm;
	double quality;
} regdata;

typedef enum { SEQ_REGULAR, SEQ_SER, SEQ_INTERNAL } sequence_type;

typedef struct ffit fits;

typedef struct sequ {
	char *seqname;
	int number;
	int selnum;
	int fixed;
	int nb_layers;
	unsigned int rx;
	unsigned int ry;
	layer_info *layers;
	int reference_image;
	imgdata *imgparam;
	regdata **regparam;
	int beg;
	int end;
	double exposure;
	int previewX[PREVIEW_NB], previewY[PREVIEW_NB];
	int previewW[PREVIEW_NB], previewH[PREVIEW_NB];
	sequence_type type;
	struct ser_struct *ser_file;
	fits **internal_fits;
	fitsfile **fptr;
	void *fd_lock;		/* omp_lock_t * */
	fits *offset;
	fits *dark;
	fits *flat;
	char *ppprefix;
	int current;
	gboolean needs_saving;
	fitted_PSF **photometry[MAX_SEQPSF];
	int reference_star;
	double reference_mag;
	double photometry_colors[MAX_SEQPSF][3];
} sequence;

struct ffit {
	unsigned int rx;
	unsigned int ry;
	int bitpix;
	int naxis;
	long naxes[3];
	WORD lo;
	WORD hi;
	float pixel_size_x, pixel_size_y;
	unsigned int binning_x, binning_y;
	char date_obs[FLEN_VALUE];
	char date[FLEN_VALUE];
	char instrume[FLEN_VALUE];
	char telescop[FLEN_VALUE];
	char observer[FLEN_VALUE];
	char bayer_pattern[FLEN_VALUE];
	double focal_length, iso_speed, exposure, aperture, ccd_temp;
	double cvf;
	double dft_norm[3];
	char dft_type[FLEN_VALUE];
	char dft_ord[FLEN_VALUE];
	unsigned int dft_rx, dft_ry;
	unsigned short min[3];
	unsigned short max[3];
	unsigned short maxi;
	unsigned short mini;
	fitsfile *fptr;
	WORD *data;
	WORD *pdata[3];
	char *header;
};

typedef struct rectangle_struct {
	int x, y, w, h;
} rectangle;

typedef enum { OPENCV_NEAREST = 0, OPENCV_LINEAR = 1, OPENCV_AREA = 2, OPENCV_CUBIC = 3, OPENCV_LANCZOS4 = 4,
	OPENCV_INTER_MAX = 7 } opencv_interpolation;

typedef int (*seq_image_filter)(sequence *seq, int nb_img, double param);

struct stacking_args;
typedef int (*stack_method)(struct stacking_args *args);

typedef enum { NO_REJEC, PERCENTILE, SIGMA, SIGMEDIAN, WINSORIZED, LINEARFIT } rejection;
typedef enum { NO_NORM, ADDITIVE, MULTIPLICATIVE, ADDITIVE_SCALING, MULTIPLICATIVE_SCALING } normalization;

typedef struct normalization_coeff {
	double *offset;
	double *mul;
	double *scale;
} norm_coeff;

struct stacking_args {
	stack_method method;
	sequence *seq;
	seq_image_filter filtering_criterion;
	double filtering_parameter;
	int nb_images_to_stack;
	int *image_indices;
	char description[100];
	const char *output_filename;
	gboolean output_overwrite;
	struct timeval t_start;
	int retval;
	int max_number_of_rows;
	double sig[2];
	rejection type_of_rejection;
	normalization normalize;
	gboolean force_norm;
};

struct registration_args;
typedef int (*registration_function)(struct registration_args *);

struct registration_args {
	registration_function func;
	sequence *seq;
	gboolean process_all_frames;
	rectangle selection;
	int layer;
	struct timeval t_start;
	int retval;
	gboolean run_in_thread;
	const gchar *prefix;
	gboolean follow_star;
	gboolean load_new_sequence;
	gboolean matchSelection;
	opencv_interpolation interpolation;
	gboolean translation_only;
	int new_total;
	imgdata *imgparam;
	regdata *regparam;
};

/* ---- the reference functions the glue calls (in Siril: the real ones; here: siril_env.c) ---- */
extern fits gfit;				/* src/core/siril.h:635-642 */
struct harness_com { int max_thread; };		/* the one cominfo field the glue reads */
extern struct harness_com com;
int seq_opened_read_region(sequence *seq, int layer, int index, WORD *buffer, const rectangle *area);
int seq_read_frame_part(sequence *seq, int layer, int index, fits *dest, const rectangle *area,
		gboolean do_photometry);
int get_thread_run(void);
/* cfitsio (Siril links the real one; here siril_env.c reads the header cards of the
 * sequence's opened files): TDOUBLE and TSTRING values */
int fits_read_key(fitsfile *fptr, int datatype, const char *keyname, void *value, char *comm, int *status);
int get_registration_layer(void);
int compute_normalization(struct stacking_args *args, norm_coeff *coeff, normalization mode);
void clearfits(fits *fit);
char *siril_log_message(const char *format, ...);
int stack_filter_all(sequence *seq, int nb_img, double any);
int stack_filter_included(sequence *seq, int nb_img, double any);

/* ---- the replacement bodies (siril_glue.c) ---- */
int stack_summing(struct stacking_args *args);
int stack_median(struct stacking_args *args);
int stack_mean_with_rejection(struct stacking_args *args);
int stack_addmax(struct stacking_args *args);
int stack_addmin(struct stacking_args *args);
int register_shift_dft(struct registration_args *args);

#endif /* SIRIL_COMPAT_H */

/*
 * sg_seqfile.cpp - Siril .seq files: the sequence description the
 * stacker and the registration read and write (readseqfile / writeseqfile,
 * src/io/seqfile.c:43-357): the S line (name, first index, images, selected, fixed length,
 * reference image), T (SER / film), L (layers), one I line per image (file number,
 * inclusion, and the cached statistics mean median sigma avgDev mad sqrtbwmv location
 * scale min max that normalisation reads) and R<layer> lines (shiftx shifty
 * rot_centre_x rot_centre_y angle fwhm quality).
 *
 * The text formats are the reference's: sscanf "%d %d %lg ..." / "%d %d %g %g %g %g %lg" on
 * read, printf "%g" on write, so statistics cached in a .seq carry six significant digits,
 * as the reference's do (normalisation coefficients computed from cached statistics see
 * the rounded values).  Host-only plumbing: no device code.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>
#include "../../include/sirilgpu.h"
#include "../../include/sirilgpu_io.h"

struct SgRegRow {
	int shiftx, shifty;
	float rot_centre_x, rot_centre_y, angle, fwhm;
	double quality;
};

struct sg_seqfile {
	std::string name;
	int beg = 0, number = 0, selnum = 0, fixed = 0, reference_image = -1;
	int type = SG_SEQFILE_REGULAR;
	int nb_layers = -1;
	std::vector<int> filenum, incl, has_stats;
	std::vector<double> stats;	/* [number][10] */
	std::vector<std::vector<SgRegRow>> reg;	/* per layer (empty: none) */
};

extern "C" void sg_seqfile_free(sg_seqfile *sf) {
	delete sf;
}

/* per-image arrays of `number` images; false when they cannot be allocated (a malformed
 * count must come back as an error code, not as an exception across the C ABI) */
static bool sf_alloc(sg_seqfile *sf, int number) {
	try {
		sf->filenum.assign(number, 0);
		sf->incl.assign(number, 0);
		sf->has_stats.assign(number, 0);
		sf->stats.assign((size_t)number * 10, 0.0);
	} catch (const std::exception &) {
		return false;
	}
	return true;
}

static bool reg_alloc(std::vector<SgRegRow> &rl, int number) {
	try {
		rl.assign(number, SgRegRow{0, 0, 0.f, 0.f, 0.f, 0.f, 0.0});
	} catch (const std::exception &) {
		return false;
	}
	return true;
}

extern "C" int sg_seqfile_read(const char *path, sg_seqfile **out) {
	if (!path || !out)
		return SG_ERR_GENERIC;
	*out = nullptr;
	std::string fn(path);
	if (fn.size() < 4 || fn.compare(fn.size() - 4, 4, ".seq") != 0)
		fn += ".seq";	/* name with or without .seq (:55-60) */
	FILE *f = fopen(fn.c_str(), "r");
	if (!f)
		return SG_ERR_READ;
	sg_seqfile *sf = new (std::nothrow) sg_seqfile();
	if (!sf) {
		fclose(f);
		return SG_ERR_SIZE;
	}
	char line[512], filename[512];
	bool allocated = false;
	int i = 0, current_layer = -1;
	int rc = SG_OK;
	while (fgets(line, 511, f)) {
		switch (line[0]) {
		case '#':
			continue;
		case 'S': {
			const char *fmt = line[2] == '\'' ? "'%511[^']' %d %d %d %d %d" : "%511s %d %d %d %d %d";
			if (sscanf(line + 2, fmt, filename, &sf->beg, &sf->number, &sf->selnum, &sf->fixed,
						&sf->reference_image) != 6 || allocated || sf->number < 1) {
				rc = SG_ERR_READ;
				goto done;
			}
			sf->name = filename;
			if (!sf_alloc(sf, sf->number)) {
				rc = SG_ERR_SIZE;
				goto done;
			}
			allocated = true;
			break;
		}
		case 'L':
			if (line[1] == ' ') {
				if (sscanf(line + 2, "%d", &sf->nb_layers) != 1 || sf->nb_layers < 1 || sf->nb_layers > 10) {
					rc = SG_ERR_READ;
					goto done;
				}
				sf->reg.assign(sf->nb_layers, std::vector<SgRegRow>());
			}
			break;
		case 'I': {
			if (!allocated || i >= sf->number) {
				rc = SG_ERR_READ;
				goto done;
			}
			double *st = &sf->stats[(size_t)i * 10];
			const int nt = sscanf(line + 2, "%d %d %lg %lg %lg %lg %lg %lg %lg %lg %lg %lg", &sf->filenum[i],
					&sf->incl[i], st, st + 1, st + 2, st + 3, st + 4, st + 5, st + 6, st + 7, st + 8, st + 9);
			if (nt == 12) {
				sf->has_stats[i] = 1;
			} else if (nt != 2) {
				rc = SG_ERR_READ;
				goto done;
			}
			++i;
			break;
		}
		case 'R': {
			current_layer = line[1] - '0';
			if (current_layer < 0 || current_layer > 9 || current_layer >= (int)sf->reg.size() || !allocated) {
				rc = SG_ERR_READ;
				goto done;
			}
			std::vector<SgRegRow> &rl = sf->reg[current_layer];
			if (rl.empty()) {
				if (!reg_alloc(rl, sf->number)) {
					rc = SG_ERR_SIZE;
					goto done;
				}
				i = 0;	/* the reference reuses the image counter (:147-150) */
			}
			if (i < sf->number) {
				SgRegRow &r = rl[i];
				const int nt = sscanf(line + 3, "%d %d %g %g %g %g %lg", &r.shiftx, &r.shifty, &r.rot_centre_x,
						&r.rot_centre_y, &r.angle, &r.fwhm, &r.quality);
				if (nt != 7) {
					if (nt == 3) {	/* old format (:158-163): the third token is dropped, the rest stays 0 */
						r.rot_centre_x = 0.0f;
					} else {
						rc = SG_ERR_READ;
						goto done;
					}
				}
				++i;
			}
			break;
		}
		case 'T':
			sf->type = line[1] == 'S' ? SG_SEQFILE_SER : (line[1] == 'A' ? SG_SEQFILE_FILM : sf->type);
			break;
		}
	}
	if (!allocated)
		rc = SG_ERR_READ;
done:
	fclose(f);
	if (rc) {
		delete sf;
		return rc;
	}
	/* the selection count is fixed to the actual value (not saved), :253-259 */
	int nbsel = 0;
	for (int k = 0; k < sf->number; k++)
		nbsel += sf->incl[k] != 0;
	sf->selnum = nbsel;
	*out = sf;
	return SG_OK;
}

extern "C" int sg_seqfile_create(const char *name, int beg, int number, int fixed, int reference_image, int type,
		int nb_layers, sg_seqfile **out) {
	if (!name || !out || number < 1 || nb_layers < 1 || nb_layers > 10)
		return SG_ERR_GENERIC;
	sg_seqfile *sf = new (std::nothrow) sg_seqfile();
	if (!sf)
		return SG_ERR_SIZE;
	sf->name = name;
	sf->beg = beg;
	sf->number = number;
	sf->fixed = fixed;
	sf->reference_image = reference_image;
	sf->type = type;
	sf->nb_layers = nb_layers;
	if (!sf_alloc(sf, number)) {
		delete sf;
		return SG_ERR_SIZE;
	}
	for (int k = 0; k < number; k++)
		sf->filenum[k] = beg + k;
	sf->incl.assign(number, 1);
	sf->selnum = number;
	sf->reg.assign(nb_layers, std::vector<SgRegRow>());
	*out = sf;
	return SG_OK;
}

extern "C" int sg_seqfile_get_info(const sg_seqfile *sf, sg_seqfile_info *info) {
	if (!sf || !info)
		return SG_ERR_GENERIC;
	memset(info, 0, sizeof *info);
	snprintf(info->name, sizeof info->name, "%s", sf->name.c_str());
	info->beg = sf->beg;
	info->number = sf->number;
	info->selnum = sf->selnum;
	info->fixed = sf->fixed;
	info->reference_image = sf->reference_image;
	info->type = sf->type;
	info->nb_layers = sf->nb_layers;
	return SG_OK;
}

extern "C" int sg_seqfile_get_images(const sg_seqfile *sf, int *filenum, int *incl, int *has_stats, double *stats) {
	if (!sf)
		return SG_ERR_GENERIC;
	for (int k = 0; k < sf->number; k++) {
		if (filenum)
			filenum[k] = sf->filenum[k];
		if (incl)
			incl[k] = sf->incl[k];
		if (has_stats)
			has_stats[k] = sf->has_stats[k];
		if (stats)
			memcpy(stats + (size_t)k * 10, &sf->stats[(size_t)k * 10], 10 * sizeof(double));
	}
	return SG_OK;
}

extern "C" int sg_seqfile_set_image(sg_seqfile *sf, int index, int filenum, int incl, const double *stats) {
	if (!sf || index < 0 || index >= sf->number)
		return SG_ERR_GENERIC;
	sf->filenum[index] = filenum;
	sf->incl[index] = incl;
	sf->has_stats[index] = stats != nullptr;
	if (stats)
		memcpy(&sf->stats[(size_t)index * 10], stats, 10 * sizeof(double));
	int nbsel = 0;
	for (int k = 0; k < sf->number; k++)
		nbsel += sf->incl[k] != 0;
	sf->selnum = nbsel;
	return SG_OK;
}

extern "C" int sg_seqfile_get_registration(const sg_seqfile *sf, int layer, int *shiftx, int *shifty,
		float *rot_centre_x, float *rot_centre_y, float *angle, float *fwhm, double *quality) {
	if (!sf || layer < 0 || layer >= (int)sf->reg.size())
		return SG_ERR_GENERIC;
	const std::vector<SgRegRow> &rl = sf->reg[layer];
	if (rl.empty())
		return 1;	/* no registration data for this layer */
	for (int k = 0; k < sf->number; k++) {
		if (shiftx)
			shiftx[k] = rl[k].shiftx;
		if (shifty)
			shifty[k] = rl[k].shifty;
		if (rot_centre_x)
			rot_centre_x[k] = rl[k].rot_centre_x;
		if (rot_centre_y)
			rot_centre_y[k] = rl[k].rot_centre_y;
		if (angle)
			angle[k] = rl[k].angle;
		if (fwhm)
			fwhm[k] = rl[k].fwhm;
		if (quality)
			quality[k] = rl[k].quality;
	}
	return SG_OK;
}

extern "C" int sg_seqfile_set_registration(sg_seqfile *sf, int layer, const int *shiftx, const int *shifty,
		const double *quality) {
	if (!sf || layer < 0 || layer >= (int)sf->reg.size() || !shiftx || !shifty)
		return SG_ERR_GENERIC;
	std::vector<SgRegRow> &rl = sf->reg[layer];
	if (!reg_alloc(rl, sf->number))
		return SG_ERR_SIZE;
	for (int k = 0; k < sf->number; k++) {
		rl[k].shiftx = shiftx[k];
		rl[k].shifty = shifty[k];
		rl[k].quality = quality ? quality[k] : 0.0;
	}
	return SG_OK;
}

/* writeseqfile (:286-357), same line formats */
extern "C" int sg_seqfile_write(const sg_seqfile *sf, const char *path) {
	if (!sf || !path || sf->name.empty())
		return SG_ERR_GENERIC;
	FILE *f = fopen(path, "w+");
	if (!f)
		return SG_ERR_READ;
	fprintf(f, "#Siril sequence file. Contains list of files (images), selection, and registration data\n");
	fprintf(f, "#S 'sequence_name' start_index nb_images nb_selected fixed_len reference_image\n");
	fprintf(f, "S '%s' %d %d %d %d %d\n", sf->name.c_str(), sf->beg, sf->number, sf->selnum, sf->fixed,
			sf->reference_image);
	if (sf->type != SG_SEQFILE_REGULAR)
		fprintf(f, "T%c\n", sf->type == SG_SEQFILE_SER ? 'S' : 'A');
	fprintf(f, "L %d\n", sf->nb_layers);
	for (int i = 0; i < sf->number; ++i) {
		if (sf->has_stats[i]) {
			const double *st = &sf->stats[(size_t)i * 10];
			fprintf(f, "I %d %d %g %g %g %g %g %g %g %g %g %g\n", sf->filenum[i], sf->incl[i], st[0], st[1],
					st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[9]);
		} else {
			fprintf(f, "I %d %d\n", sf->filenum[i], sf->incl[i]);
		}
	}
	for (int j = 0; j < (int)sf->reg.size(); j++) {
		if (sf->reg[j].empty())
			continue;
		for (int i = 0; i < sf->number; ++i) {
			const SgRegRow &r = sf->reg[j][i];
			fprintf(f, "R%d %d %d %g %g %g %g %g\n", j, r.shiftx, r.shifty, r.rot_centre_x, r.rot_centre_y,
					r.angle, r.fwhm, r.quality);
		}
	}
	return fclose(f) == 0 ? SG_OK : SG_ERR_READ;
}

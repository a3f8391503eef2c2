/* pfe_io.h — native PHCX / SUPERB-PHCX reader and batch packer of libpfe.so (host code).
 *
 * Replaces the per-candidate file decoding of the reference (paths relative to
 * PulsarFeatureExtractor/src/):
 *   Candidate.py:141-150          file-type dispatch (".gz" in the name -> HTRU PHCX, else SUPERB)
 *   PHCXFile.py:80-186            gzip + minidom load, Profile hex decode (section 1)
 *   SUPERBPHCXFile.py:80-186      plain XML load, Profile hex decode (section 0)
 *   PHCXOperations.py:81-112      BestValues scalars (BaryPeriod*1000, Snr, Dm, Width)
 *   PHCXOperations.py:121-259     DmIndex parse (:172-183), DataBlock decode, dm_curve reduction
 *   PHCXOperations.py:263-297     getDM_FFT DataBlock hex decode (Lyon DM array: section 0, :538)
 *   PHCXOperations.py:305-383     SubBands + hexToDec
 * Files are parsed by a pool of host threads; hex text is decoded with the reference's rule
 * (skip '\n' only, consume aligned pairs, int(pair, 16) semantics incl. surrounding whitespace
 * and a sign, stop at the first pair that does not parse).  A file that the native reader
 * cannot reproduce exactly (decoded values outside 0..255, malformed text) gets a non-zero
 * status; the host then falls back to its Python parser for that file.
 */
#ifndef PFE_IO_H
#define PFE_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-file status (pfe_phcx_info.status) */
#define PFE_IO_OK 0
#define PFE_IO_ERR_OPEN 1  /* cannot open / read the file (IOError) */
#define PFE_IO_ERR_GZIP 2  /* corrupt gzip stream */
#define PFE_IO_ERR_XML 3   /* a required element is missing (IndexError) */
#define PFE_IO_ERR_VALUE 4 /* a scalar / DmIndex token / attribute does not parse (ValueError) */
#define PFE_IO_ERR_RANGE 5 /* decoded values outside 0..255 (signed pairs such as "-1") */
#define PFE_IO_ERR_SHAPE 6 /* SubBands length != nSub * nBins (reshape error) */

/* fields for pfe_phcx_fetch */
#define PFE_PHCX_PROFILE 0    /* uint8[lp]        scored-section Profile              */
#define PFE_PHCX_LYON_DM 1    /* uint8[ld]        DataBlock of section 0              */
#define PFE_PHCX_SUBBANDS 2   /* uint8[nsub*lsb]  scored-section SubBands, row-major  */
#define PFE_PHCX_DM_CURVE 3   /* double[ndm]      reduced DM curve (max of 127/128)    */
#define PFE_PHCX_FIT_BLOCK 4  /* uint8[lfit]      scored-section DataBlock            */

typedef struct {
  int32_t status;  /* PFE_IO_* */
  int32_t superb;  /* 1: SUPERB (plain XML, section 0); 0: HTRU PHCX (gzip, section 1) */
  int32_t section; /* scored XML section */
  int32_t lp;      /* profile bins */
  int32_t nsub;    /* sub-bands */
  int32_t lsb;     /* bins per sub-band */
  int32_t ndm;     /* reduced DM-curve points = lfit / 128 */
  int32_t reserved;
  int64_t ld;      /* Lyon DM array length */
  int64_t lfit;    /* scored DataBlock length (length_all) */
  /* PFE_NSCAL layout of pfe_bates_in.scal: period_ms, snr, dm, width, dm_start, dm_end,
     length_all, 0 */
  double scal[8];
} pfe_phcx_info;

typedef struct pfe_phcx_batch pfe_phcx_batch;

/* Parse n files with nthreads host threads (<= 0: all hardware threads).  mode: -1 decides
   per file by name like Candidate.py:141-150, 0 = HTRU PHCX, 1 = SUPERB.  Returns PFE_OK or
   PFE_EINVAL; per-file problems are reported in the file's info.status. */
int pfe_phcx_parse(const char* const* paths, int64_t n, int32_t mode, int32_t nthreads,
                   pfe_phcx_batch** out);
int64_t pfe_phcx_count(const pfe_phcx_batch* b);
int pfe_phcx_info_get(const pfe_phcx_batch* b, int64_t i, pfe_phcx_info* info);
/* copy one decoded field of file i into dst (capacity in elements); PFE_EINVAL if it does
   not fit or the file failed */
int pfe_phcx_fetch(const pfe_phcx_batch* b, int64_t i, int32_t field, void* dst,
                   int64_t capacity);
/* Gather rows (file indices) into dense, caller-owned arrays for pfe_bates22 / pfe_lyon8_u8:
   prof[nrows][prof_stride] (lp bytes used), lyon_dm[nrows][dm_stride] (ld bytes used),
   sub[nrows][sub_stride] (nsub*lsb used), dmcurve[nrows][dmc_stride] (ndm used),
   scal[nrows][8].  Any output may be NULL.  Every row must be a parsed file whose lengths
   fit the strides (else PFE_EINVAL, nothing partial is promised). */
int pfe_phcx_pack(const pfe_phcx_batch* b, const int64_t* rows, int64_t nrows,
                  int32_t nthreads, uint8_t* prof, int64_t prof_stride, uint8_t* lyon_dm,
                  int64_t dm_stride, uint8_t* sub, int64_t sub_stride, double* dmcurve,
                  int64_t dmc_stride, double* scal);
void pfe_phcx_free(pfe_phcx_batch* b);
/* Every file's info in one call: out[0 .. count) (capacity >= pfe_phcx_count(b), else
   PFE_EINVAL).  Replaces a per-file pfe_phcx_info_get loop on the batched product path. */
int pfe_phcx_info_all(const pfe_phcx_batch* b, pfe_phcx_info* out, int64_t capacity);

/* Score rows as text, the way DataProcessor writes them:
     style 0  storeScore      (DataProcessor.py:321-325)  "<name>,v1,...,vw\n"
     style 1  storeScoreARFF  (DataProcessor.py:421-425)  "v1,...,vw,?%<name>\n"
     style 2  outputScores    (DataProcessor.py:443-446)  "v1,...,vw\n" (name unused)
   Every value is Python 2.7's str(float): '%.12g', ".0" appended when the text has no '.',
   'e' or 'n'; NaN -> "nan", +-inf -> "inf" / "-inf"; then, as the reference does on the
   joined line, every "nan" and afterwards every "inf" becomes "0" (in the name too).
   names: the n names back to back in `name_blob`, name i = [name_off[i], name_off[i+1]).
   vals: row i at vals + i*stride (width doubles).  Rows with skip[i] != 0 are left out
   (skip may be NULL).  The text goes to buf (capacity cap); *len receives its length.
   PFE_EINVAL if it does not fit (cap >= sum(name lengths) + n*(24*width + 8) always does). */
int pfe_format_rows(const char* name_blob, const int64_t* name_off, const double* vals,
                    int64_t n, int32_t width, int64_t stride, int32_t style,
                    const uint8_t* skip, int32_t nthreads, char* buf, int64_t cap,
                    int64_t* len);

#ifdef __cplusplus
}
#endif

#endif /* PFE_IO_H */

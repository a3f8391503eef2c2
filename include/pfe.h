/*
 * pfe.h — C-ABI of libpfe.so, the MI355X (gfx950) batched pulsar-candidate feature engine.
 *
 * This is the drop-in boundary for the per-candidate score path of
 * scienceguyrob/PulsarFeatureExtractor (ScoreGenerator.py).  The reference computes one
 * candidate at a time in Python; every entry point here is the BATCHED equivalent of one
 * reference interface, taking row-major candidate arrays (plain pointers + sizes, no
 * framework types) and writing one row of fp64 scores per candidate.
 *
 * Interfaces replaced (reference paths relative to PulsarFeatureExtractor/src/):
 *   pfe_lyon8_u8   <- PHCXFile.computeProfileStatScores          PHCXFile.py:320-349
 *                     + PHCXFile.computeDMCurveStatScores         PHCXFile.py:351-379
 *                     (concatenated as in DataProcessor.dmprof    DataProcessor.py:884-886;
 *                      SUPERBPHCXFile.py has identical bodies at the same lines)
 *   pfe_lyon8_f64  <- the same two functions on float profiles (PFDFile.py:522-583)
 *   pfe_bates22    <- PHCXFile.compute                            PHCXFile.py:383-409
 *                     (score groups 1-4 :413, 5-11 :475, 12-15 :547, 16-19 :589, 20-22 :633)
 *
 * Conventions
 *   - One handle per (device, stream).  Calls on one handle are serialised by the caller;
 *     different handles may be used concurrently from different threads.
 *   - Caller owns all input/output buffers.  With PFE_FLAG_DEVICE_PTRS the pointers are
 *     device (HBM) pointers and the call is asynchronous on the handle's stream (no host
 *     sync); without it they are host pointers and the library stages them through
 *     per-handle device scratch, returning when the outputs are back on the host.
 *   - The 22-score calls run their independent score groups on two side streams the handle
 *     owns; they start after the work already queued on the handle's stream and are joined
 *     back into it (events) before the call returns, so callers only ever see one stream.
 *   - Raw IEEE values are returned (NaN/inf included).  NaN/inf -> "0" replacement is the
 *     writer's job, as in DataProcessor.storeScore (DataProcessor.py:321-325).
 *   - Return value: 0 = OK, otherwise a PFE_E* code; the text is in pfe_last_error().
 *   - There is NO CPU backend: pfe_create(-1, ...) fails.  The CPU restatement used for
 *     parity testing lives in oracle/ and is not part of this library.
 */
#ifndef PFE_H_
#define PFE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFE_ABI_VERSION 1

/* return codes */
#define PFE_OK 0
#define PFE_EINVAL 1   /* bad argument (null pointer, negative size, unsupported layout) */
#define PFE_EDEVICE 2  /* HIP runtime failure (allocation, launch, copy) */
#define PFE_ENODEV 3   /* no such device / no GPU present */

/* flags */
#define PFE_FLAG_DEVICE_PTRS 0x1u /* all array arguments are device pointers */

/* Per-candidate status bits (pfe_bates22).  A non-zero status means the reference would
 * have raised inside Candidate.calculateScores and DataProcessor would have logged the
 * candidate to CandidateErrorLog.txt and dropped its row (DataProcessor.py:517-523). */
#define PFE_ST_SINE_FAIL      0x001u /* scores 1-4 raised            (PHCXFile.py:467-470) */
#define PFE_ST_GAUSS_FAIL     0x002u /* scores 5-11 raised           (PHCXFile.py:540-543) */
#define PFE_ST_DMFIT_FAIL     0x004u /* scores 16-19 raised          (PHCXFile.py:626-629) */
#define PFE_ST_SUBBAND_FAIL   0x008u /* scores 20-22 raised          (PHCXFile.py:665-668) */
#define PFE_ST_UNSUPPORTED    0x010u /* outside the shapes this build scores (a histogram with
                                        more than 16384 Freedman-Diaconis bins).  Unreachable
                                        for byte (PHCX) profiles of up to 32768 bins: their
                                        non-zero IQR is a multiple of 0.25, so the bin count
                                        is at most 510 n^(1/3); or, in pfe_bates22, a
                                        sub-band shape beyond nsub 65536 x nBins 16384 --
                                        the other groups' scores are still computed).  The
                                        row is not scored.  pfe_bates22 refuses the whole
                                        call (PFE_EINVAL) when nsub * nBins > 2^24 bytes
                                        per candidate, so the per-row mark is reached by
                                        nsub > 65536 with nBins < 256 or nBins > 16384
                                        with nsub < 1024 */
#define PFE_ST_DGF_INDEXERROR 0x100u /* informational: double-Gaussian IndexError path taken,
                                        s10=s11=1e6 (ProfileOperations.py:762-764) */
#define PFE_ST_FAIL_MASK      0x0FFu

typedef struct pfe_handle pfe_handle;

/* Query the ABI version compiled into the library. */
int pfe_abi_version(void);

/* Number of visible GPUs (0 when none); never fails. */
int pfe_device_count(void);

/* Create a handle bound to GPU `device` (>= 0) and its own non-blocking stream. */
int pfe_create(int device, pfe_handle** out);
void pfe_destroy(pfe_handle* h);

/* Text of the last error on this handle (or of the last failed pfe_create when h is NULL). */
const char* pfe_last_error(const pfe_handle* h);

/* Launch subsequent work on `hip_stream` (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL selects the HIP default (null) stream.  A new handle starts on its own non-blocking
 * stream.  The library never destroys a stream it did not create. */
int pfe_set_stream(pfe_handle* h, void* hip_stream);
/* Block until all work queued on the handle's stream has finished. */
int pfe_synchronize(pfe_handle* h);

/* ---------------------------------------------------------------------------------------
 * Handle options (A/B and verification switches).  The defaults are the product
 * configuration; the library never reads the process environment, so only an explicit
 * pfe_set_option changes what a handle computes.  Options marked (bits) change the last
 * bits of the LM-fitted scores (the m-sums are ordered differently); all others give
 * identical results and only change the schedule.
 *   PFE_OPT_SOLVER       (bits) LM solver of the 22-score kernels: PFE_SOLVER_POOLED
 *                        (default; pooled group engine for <= 256 bins -- 16-lane groups up
 *                        to 128 bins, 32-lane groups above -- batched beyond),
 *                        PFE_SOLVER_BATCHED (one wave owns 32 fits), or
 *                        PFE_SOLVER_WAVE (one wave per fit; bit-identical to BATCHED)
 *   PFE_OPT_SERIAL       1: the independent score groups run in order on the handle's
 *                        stream instead of on its two side streams (default 0)
 *   PFE_OPT_HANDOVER     0: re-evaluate the residuals after an accepted LM step instead of
 *                        handing the trial's residuals over (default 1)
 *   PFE_OPT_GSLOTS       fit slots per pooled wave, 1..32 (0 = sized from n; default 0)
 *   PFE_OPT_LYON8_BLOCKS grid cap of the Lyon-8 kernels (default 131072)
 *   PFE_OPT_LYON8_BURST  candidate groups per wave step of the Lyon-8 kernel: 1, 2 or 4
 *                        (default 2)
 *   PFE_OPT_PFD_WAVES    waves per fold of the PFD preprocessing kernel: 4 (default) or 1
 *   PFE_OPT_LYON8_DM     Lyon-8 kernel for DataBlock-length DM rows (PHCX nDM x 128 bytes):
 *                        0 = lyon8_u8_dm, skew / kurt from fp64 d^3 / d^4 sums (default);
 *                        1 = the round-3 kernels; 2 = lyon8_u8_dm with exact integer power
 *                        sums.  Mean and std are numpy's bits with every option; skew / kurt
 *                        may differ in the last bits
 *   PFE_OPT_PFD_SPLIT    PFD preprocessing: 1 = the folds' part sums streamed by their own kernel
 *                        on a side stream while the sweep kernel works on the previous chunk,
 *                        0 = one fused kernel (default; same bits)
 *   PFE_OPT_LYON8_DM_SPLIT  1 (default): the last numpy chunk of a DataBlock row with <= 32
 *                        leaves is summed by 2, 4 or 8 lanes per leaf, each taking some of the
 *                        leaf's 8 chains (the tri form's 128-byte leaves over the idle lane of
 *                        their quad), and one-chunk rows of 17-32 leaves are taken two per
 *                        wave; 2: the chain splits only; 0: one lane per leaf.  Mean and std
 *                        the same bits with every value, skew / kurt within 1e-12
 * Returns PFE_EINVAL for an unknown option or an out-of-range value.
 * --------------------------------------------------------------------------------------- */
#define PFE_OPT_SOLVER 1
#define PFE_OPT_SERIAL 2
#define PFE_OPT_HANDOVER 3
#define PFE_OPT_GSLOTS 4
#define PFE_OPT_LYON8_BLOCKS 5
#define PFE_OPT_LYON8_BURST 6
#define PFE_OPT_PFD_WAVES 7
#define PFE_OPT_LYON8_DM 8
#define PFE_OPT_PFD_SPLIT 9
#define PFE_OPT_LYON8_DM_SPLIT 10
#define PFE_SOLVER_POOLED 0
#define PFE_SOLVER_BATCHED 1
#define PFE_SOLVER_WAVE 2
int pfe_set_option(pfe_handle* h, int32_t option, int64_t value);
int pfe_get_option(const pfe_handle* h, int32_t option, int64_t* value);

/* Pinned (page-locked) host memory.  Host-pointer calls DMA pinned caller buffers in place
 * (chunked, with the copies of one chunk overlapping the kernel of another); pageable
 * buffers are staged through the handle's own pinned ring by the calling thread.  A
 * producer that writes candidate rows straight into pfe_host_alloc memory (e.g.
 * pfe_phcx_pack) therefore skips that staging copy.  Not tied to a handle. */
int pfe_host_alloc(size_t bytes, void** out);
void pfe_host_free(void* p);

/* ---------------------------------------------------------------------------------------
 * 8 Lyon features.
 *   prof : n rows of lp uint8 bins (PHCX 02X-decoded profile), row r at prof + r*prof_stride
 *   dm   : n rows of ld uint8 values (PHCX DataBlock of section 0), row r at dm + r*dm_stride
 *   out  : n x 8 fp64, row-major, per candidate
 *          [prof_mean, prof_std, prof_skew, prof_kurt, dm_mean, dm_std, dm_skew, dm_kurt]
 *          std is ddof=0; skew is the biased g1 and kurt the biased Fisher g2 of
 *          scipy.stats; both are NaN when the row has zero variance (scipy >= 1.9).
 *   status : may be NULL; set to 0 for every row (the 8-feature path has no failure mode).
 * Requires lp >= 1, ld >= 1, strides >= row lengths.
 * --------------------------------------------------------------------------------------- */
int pfe_lyon8_u8(pfe_handle* h, const uint8_t* prof, int64_t prof_stride, int32_t lp,
                 const uint8_t* dm, int64_t dm_stride, int32_t ld, int64_t n, double* out,
                 uint32_t* status, uint32_t flags);

/* Same with fp64 rows (PFD profiles are float; PFDFile.py:522-583).  Two-pass fp64
 * moments, as numpy/scipy compute them. */
int pfe_lyon8_f64(pfe_handle* h, const double* prof, int64_t prof_stride, int32_t lp,
                  const double* dm, int64_t dm_stride, int32_t ld, int64_t n, double* out,
                  uint32_t* status, uint32_t flags);

/* ---------------------------------------------------------------------------------------
 * 22 Bates scores (PHCX / SUPERB PHCX).
 *   prof    : n x lp uint8 profile (Profile of the scored section)
 *   sub     : n x nsub x lsb uint8 sub-bands (SubBands of the scored section)
 *   dmcurve : n x ndm fp64 reduced DM curve (PHCXOperations.dm_curve of that section's
 *             DataBlock: max over the first 127 of every 128 values); point k sits at
 *             DM = dm_start + (128k - 1) * |dm_start - dm_end| / length_all  (:196)
 *   scal    : n x PFE_NSCAL fp64 per-candidate scalars (layout below)
 *   out     : n x 22 fp64 in reference score order (score 1 in column 0)
 *   status  : n x uint32 PFE_ST_* bits (required)
 * Strides are in elements and equal the row length (dense rows).
 * --------------------------------------------------------------------------------------- */
#define PFE_NSCAL 8
#define PFE_SCAL_PERIOD_MS 0 /* BaryPeriod * 1000            (PHCXOperations.py:109) */
#define PFE_SCAL_SNR 1       /* Snr                            (:107) */
#define PFE_SCAL_DM 2        /* Dm                             (:108) */
#define PFE_SCAL_WIDTH 3     /* Width                          (:110) */
#define PFE_SCAL_DM_START 4  /* float(DmIndex token[1])        (:172-182) */
#define PFE_SCAL_DM_END 5    /* float(DmIndex last token)      (:182) */
#define PFE_SCAL_LENGTH_ALL 6 /* len(decoded DataBlock)        (:168) */
#define PFE_SCAL_RESERVED 7

typedef struct pfe_bates_in {
  const uint8_t* prof;  /* n x lp */
  int32_t lp;
  const uint8_t* sub;   /* n x nsub x lsb */
  int32_t nsub;
  int32_t lsb;
  const double* dmcurve; /* n x ndm */
  int32_t ndm;
  const double* scal;   /* n x PFE_NSCAL */
  int64_t n;
} pfe_bates_in;

int pfe_bates22(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                uint32_t flags);

/* Sub-band scores alone (scores 20-22):
 *   pfe_subband3 <- PHCXOperations.getSubbandParameters          PHCXOperations.py:305-349
 *                   (getSubband_scores ProfileOperations.py:1585-1686, getProfileCorr
 *                    PHCXOperations.py:387-415)
 * Reads prof, sub and scal[PFE_SCAL_WIDTH] of `in` (dmcurve/ndm are ignored and may be
 * NULL/0); out = n x 3 fp64 [RMS of sub-band peak positions, mean pairwise correlation,
 * sum of profile correlations > 0.0055]; status bits PFE_ST_SUBBAND_FAIL where the
 * reference raises (boxcar width <= 0 or > nBins, every pair NaN, lp != lsb).
 * Any nsub in [1, 65536] and lsb in [1, 16384] (lp up to 16384 here): nsub 2-256 with
 * nsub * (lsb + 1) <= 32768 on chip, every other shape through global scratch of the handle. */
int pfe_subband3(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                 uint32_t flags);

/* One score group of the chain alone: the batched form of one method of the reference's
 * second plug-in class, ProfileOperationsInterface (ProfileOperationsInterface.py:69-130),
 * as PHCXOperations implements it.  `in` as for pfe_bates22, but only the arrays a group
 * reads are used (the others may be NULL / 0); the same kernels, so every value is the bits
 * the group's columns of pfe_bates22 hold; status carries that group's failure bit only.
 *   pfe_sinusoid4 <- getSinusoidFittings(profile)        ProfileOperations.py:190-376
 *                    reads prof; out n x 4 = s1-s4 (pfe_bates22 columns 0-3)
 *   pfe_gauss7    <- getGaussianFittings(profile)        ProfileOperations.py:595-770
 *                    reads prof; out n x 7 = s5-s11 (columns 4-10)
 *   pfe_params4   <- getCandidateParameters(data, sec)   PHCXOperations.py:81-112
 *                    reads scal; out n x 4 = [period_ms, snr, dm, width] as the method
 *                    returns them (PHCXFile applies filterScore(13/14) for s13/s14)
 *   pfe_dmfit4    <- getDMFittings(data, sec)            PHCXOperations.py:121-233
 *                    reads dmcurve, scal; out n x 4 = [peak, |1 - Prop|, Shift, chi_theo]:
 *                    the method's signed Shift (s18 = filterScore(18, Shift) = |Shift|) */
int pfe_sinusoid4(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                  uint32_t flags);
int pfe_gauss7(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
               uint32_t flags);
int pfe_params4(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                uint32_t flags);
int pfe_dmfit4(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
               uint32_t flags);

/* ---- PFD (PRESTO fold) files: preprocessing + Lyon features -------------------------
 * pfe_pfd_dmprof <- what a freshly loaded PFDFile computes for the dmprof path
 *   dedisperse (PFDFile.py:330-374) at the best DM, getprofile + scale (:256-310),
 *   plot_chi2_vs_DM(dms[0], dms[-1]) (:378-423, 100 DMs, float32),
 *   computeProfileStatScores (:522-551) and computeDMCurveStatScores (:553-583).
 * Inputs per candidate: the fold's sub-integration profiles profs[npart][nsub][proflen],
 * the sub-band centre frequencies (PFDFile.py:222-226) and the scalars below (from the
 * file header: best DM, fold_p1 * proflen, (profs/proflen).sum() of the file as read,
 * the summed prof_var foldstats, dms[0], dms[-1] and numdms).
 * Outputs (each may be NULL): profile[n][proflen] (0..255 fp64, also the --profile bins of
 * PFDFile.computeProfileScores :479-492), chis[n][PFE_PFD_NDM] (the float32 DM curve),
 * lyon8[n][8] = [profile mean, std, skew, kurt, DM-curve mean, std, skew, kurt].
 * status[i] = PFE_ST_PFD_DMCURVE_FAIL when numdms == 1 (the reference raises on dms[0]). */
#define PFE_PFD_NSCAL 8
#define PFE_PFD_BESTDM 0
#define PFE_PFD_BINSPERSEC 1
#define PFE_PFD_AVGPROF 2
#define PFE_PFD_VARPROF 3
#define PFE_PFD_DM_LO 4
#define PFE_PFD_DM_HI 5
#define PFE_PFD_NUMDMS 6
#define PFE_PFD_BARY_P1 7 /* bary_p1 (s; the 22-score path: period = bary_p1 * 1000) */
#define PFE_PFD_NDM 100
#define PFE_ST_PFD_DMCURVE_FAIL 0x020u

typedef struct pfe_pfd_in {
  const double* profs;    /* n x npart x nsub x proflen */
  const double* subfreqs; /* n x nsub */
  const double* scal;     /* n x PFE_PFD_NSCAL */
  int32_t npart, nsub, proflen;
  int64_t n;
} pfe_pfd_in;

int pfe_pfd_dmprof(pfe_handle* h, const pfe_pfd_in* in, double* profile, float* chis,
                   double* lyon8, uint32_t* status, uint32_t flags);

/* pfe_pfd_bates22 <- PFDFile.compute (PFDFile.py:587-613): the 22 scores of each fold in the
 * reference's order -- ProfileOperations' sinusoid and Gaussian fits on the 0..255 float
 * profile (s1-s11), PFDOperations.getCandidateParameters (s12-s15, PFDOperations.py:93-233),
 * getDMFittings (s16-s19, the clamped 4-parameter fit to the chi^2-vs-DM curve, :274-393) and
 * getSubbandParameters over the dedispersed sub-band profiles (s20-s22, :401-466).
 * Same inputs as pfe_pfd_dmprof (scal[PFE_PFD_BARY_P1] is used); out[n][22]; status bits as
 * pfe_bates22 (PFE_ST_DMFIT_FAIL when numdms == 1).  LDS-resident limit as pfe_pfd_dmprof. */
int pfe_pfd_bates22(pfe_handle* h, const pfe_pfd_in* in, double* out, uint32_t* status,
                    uint32_t flags);

#ifdef __cplusplus
}
#endif

#endif /* PFE_H_ */

// bates22.hip — host launcher of the 22-score pipeline (PHCXFile.compute, PHCXFile.py:383-409).
//
// Score groups run as separate kernels on the caller's stream, in the reference's group
// order; each writes its own output columns and ORs its failure bit into status[c]:
//   k_sine (s1-s4) -> k_ghist (+ k_ghist<BIG> for wide histograms) -> k_gt1 (s8,s9)
//   -> k_gdg (s10,s11) -> k_dmfit (s12-s19) -> k_subband (s20-s22)
#include <cmath>

#include "bates_common.h"

namespace pfe {

hipError_t launch_sine(const BatesArgs& a, hipStream_t st);
hipError_t launch_gauss(const BatesArgs& a, hipStream_t st);
hipError_t launch_dmfit(const BatesArgs& a, hipStream_t st);
hipError_t launch_subband(const BatesArgs& a, hipStream_t st);
size_t subband_work_bytes(int64_t n, int nsub, int lsb);

static int device_cus() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      cus = v;
  }
  return cus;
}

// Fits per wave of the batched kernels: as many as fit the LDS state (32), but few enough
// that the grid holds ~4 waves for every one of (CUs x 16) wave slots -- each wave runs its
// fits one after another, so a batch of fewer waves than slots finishes with its slowest wave
static int blm_fits_per_wave(int64_t n, int cus) {
  const int64_t f = n / ((int64_t)cus * 64);
  return (int)(f < 4 ? 4 : f > BLM_FPW ? BLM_FPW : f);
}

// Fit slots per wave of the pooled kernels (lm_group.h): a wave works its slots in groups of
// 4 and runs lmpar one slot per lane, so it wants many; but n / slots waves should still
// cover the chip's wave slots (CUs x 8) -- the handle option PFE_OPT_GSLOTS overrides
static int glm_slots(int64_t n, int cus, int fixed) {
  if (fixed > 0) return fixed > GLM_FPW ? GLM_FPW : fixed;
  const int64_t f = n / ((int64_t)cus * 8);
  return (int)(f < 4 ? 4 : f > GLM_FPW ? GLM_FPW : f);
}

// persistent waves of the batched and pooled kernels: enough to fill every CU (8 waves
// each), never more than there are batches
static int persistent_waves(int64_t n) {
  const int cus = device_cus();
  const int fpw = blm_fits_per_wave(n, cus);
  const int64_t batches = (n + fpw - 1) / fpw;
  const int64_t w = (int64_t)cus * 8;
  return (int)(batches < w ? (batches > 0 ? batches : 1) : w);
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// hand-over regions (lm_group.h HandOver) of the three chains: waves x slots x K x group
// lanes (16; 32 for the profile fits of > 128 bins); the Gaussian chain runs a.pwaves waves,
// the DM and sine kernels pool_grid(a, 3)
static int64_t hand_waves(int64_t n, int region) {
  const int64_t cap = (int64_t)device_cus() * (region == HAND_GAUSS ? 8 : 12);
  return n < 1 ? 1 : n < cap ? n : cap;
}
static size_t hand_bytes(int64_t n, int region, int lp) {
  const int k = region == HAND_GAUSS ? HAND_K_GAUSS : region == HAND_DM ? HAND_K_DM : HAND_K_SINE;
  const int slots = region == HAND_GAUSS ? GDG8_FPW : GLM_FPW;  // the Gaussian chain's widest pool
  return (size_t)hand_waves(n, region) * slots * k * glm_group_lanes(lp) * sizeof(double);
}

// waves of k_ghist_wide (each with a WIDE_SLAB_BYTES = 720 KB scratch slab): one per 64
// candidates up to 256, so a small batch does not carry 184 MB of slabs for a queue that is
// usually empty, and a large one still drains a big queue (low-noise data) in parallel
static int wide_waves(int64_t n) {
  const int64_t w = n / 64;
  return (int)(w < 1 ? 1 : w > 256 ? 256 : w);
}

// workspace layout: [GaussWS x n][counters][hand-over regions][wide queue][wide slabs]
// [per-wave scratch] (bates_setup) then, for sub-band shapes the LDS kernels do not hold,
// the any-shape sub-band kernel's slabs
static size_t bates22_core_bytes(const pfe_bates_in* in) {
  size_t hb = 0;
  for (int r = 0; r < 3; ++r) hb += align256(hand_bytes(in->n, r, in->lp));
  return 256 + align256((size_t)in->n * sizeof(GaussWS)) +
         align256(BATES_NCOUNTERS * sizeof(unsigned)) + hb +
         align256((size_t)in->n * sizeof(int)) + (size_t)wide_waves(in->n) * WIDE_SLAB_BYTES +
         (size_t)persistent_waves(in->n) * gdg_wave_scratch_doubles(in->lp) * sizeof(double);
}
size_t bates22_workspace_bytes(const pfe_bates_in* in) {
  const size_t sw = subband_work_bytes(in->n, in->nsub, in->lsb);
  return bates22_core_bytes(in) + (sw ? 256 + align256(sw) : 0);
}

__global__ void k_clear_internal(uint32_t* status, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) status[i] &= 0xFFFFu;
}

void launch_clear_internal(uint32_t* status, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_clear_internal, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     status, n);
}

// workspace pointers, batching parameters and the Freedman-Diaconis constants of a chain
// over n candidates of lp bins (work: bates22_workspace_bytes)
void bates_setup(BatesArgs& a, int64_t n, int lp, void* work, const Options& o) {
  char* wb = (char*)(((uintptr_t)work + 255) & ~(uintptr_t)255);
  a.ws = (GaussWS*)wb;
  wb += align256((size_t)n * sizeof(GaussWS));
  a.counters = (unsigned*)wb;
  wb += align256(BATES_NCOUNTERS * sizeof(unsigned));
  const bool ho = o.handover != 0;
  for (int r = 0; r < 3; ++r) {
    a.hand[r] = ho ? (double*)wb : nullptr;
    wb += align256(hand_bytes(n, r, lp));
  }
  a.wide_list = (int*)wb;
  wb += align256((size_t)n * sizeof(int));
  a.wide_scr = (double*)wb;
  a.wide_waves = wide_waves(n);
  wb += (size_t)a.wide_waves * WIDE_SLAB_BYTES;
  a.sub_work = nullptr;  // set by the 22-score launcher, which knows the sub-band shape
  a.raw_dm = 0;
  a.wscr = (double*)wb;
  a.pwaves = persistent_waves(n);
  a.fpw = blm_fits_per_wave(n, device_cus());
  a.gslots = glm_slots(n, device_cus(), o.gslots);
  a.solver = o.solver;
  a.cus = device_cus();
  a.lp = lp;
  a.n = n;
  // Python evaluates pow(len(data), -0.3333333) with the C library; so does this host code
  a.c_lp = std::pow((double)lp, -0.3333333);
  a.c_lp1 = std::pow((double)(lp - 1), -0.3333333);
}

// fork the three independent score groups onto the handle's side streams (false: serial,
// when the handle has none or its PFE_OPT_SERIAL option is set)
bool fork_begin(const Fork* fk, hipStream_t st) {
  if (!fk || !fk->side[0] || fk->serial) return false;
  if (hipEventRecord(fk->ev[0], st) != hipSuccess) return false;
  return hipStreamWaitEvent(fk->side[0], fk->ev[0], 0) == hipSuccess &&
         hipStreamWaitEvent(fk->side[1], fk->ev[0], 0) == hipSuccess;
}
hipError_t fork_end(const Fork* fk, hipStream_t st) {
  hipError_t e;
  if ((e = hipEventRecord(fk->ev[1], fk->side[0])) != hipSuccess) return e;
  if ((e = hipEventRecord(fk->ev[2], fk->side[1])) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(st, fk->ev[1], 0)) != hipSuccess) return e;
  return hipStreamWaitEvent(st, fk->ev[2], 0);
}

// The score groups `groups` (BG_*) of the chain, each into its own columns of out (n x 22);
// status gets the failure bits of those groups only.  raw_dm: getDMFittings' signed shift in
// column 17 (the per-group entry point pfe_dmfit4) instead of the 22-score vector's |shift|.
hipError_t launch_bates_groups(const pfe_bates_in* in, double* out, uint32_t* status, void* work,
                               size_t work_bytes, hipStream_t st, const Fork* fk,
                               const Options& o, unsigned groups, bool raw_dm) {
  if (work_bytes < bates22_workspace_bytes(in)) return hipErrorInvalidValue;
  BatesArgs a;
  bates_setup(a, in->n, in->lp, work, o);
  a.raw_dm = raw_dm ? 1 : 0;
  if (subband_work_bytes(in->n, in->nsub, in->lsb))
    a.sub_work = (void*)(((uintptr_t)work + bates22_core_bytes(in) + 255) & ~(uintptr_t)255);
  a.prof = in->prof;
  a.fprof = nullptr;
  a.lp = in->lp;
  a.sub = in->sub;
  a.nsub = in->nsub;
  a.lsb = in->lsb;
  a.dmcurve = in->dmcurve;
  a.ndm = in->ndm;
  a.scal = in->scal;
  a.n = in->n;
  a.out = out;
  a.status = status;
  hipError_t e = hipMemsetAsync(status, 0, (size_t)in->n * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(out, 0, (size_t)in->n * 22 * sizeof(double), st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.counters, 0, BATES_NCOUNTERS * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  if (groups == BG_ALL && fork_begin(fk, st)) {
    if ((e = launch_gauss(a, fk->side[0])) != hipSuccess) return e;
    if ((e = launch_dmfit(a, fk->side[1])) != hipSuccess) return e;
    if ((e = launch_subband(a, fk->side[1])) != hipSuccess) return e;
    if ((e = launch_sine(a, st)) != hipSuccess) return e;
    if ((e = fork_end(fk, st)) != hipSuccess) return e;
  } else {
    if ((groups & BG_SINE) && (e = launch_sine(a, st)) != hipSuccess) return e;
    if ((groups & BG_GAUSS) && (e = launch_gauss(a, st)) != hipSuccess) return e;
    if ((groups & BG_DM) && (e = launch_dmfit(a, st)) != hipSuccess) return e;
    if ((groups & BG_SUB) && (e = launch_subband(a, st)) != hipSuccess) return e;
  }
  launch_clear_internal(status, in->n, st);
  return hipGetLastError();
}

hipError_t launch_bates22(const pfe_bates_in* in, double* out, uint32_t* status, void* work,
                          size_t work_bytes, hipStream_t st, const Fork* fk, const Options& o) {
  return launch_bates_groups(in, out, status, work, work_bytes, st, fk, o, BG_ALL, false);
}

}  // namespace pfe

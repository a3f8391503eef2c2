// capi.hip — extern "C" boundary of libpfe.so (declared in include/pfe.h).
//
// Owns: the per-handle HIP streams, device scratch, the pinned staging ring of the chunked
// host-pointer path, the handle options and the argument validation that mirrors the
// reference's failure behaviour.  No CPU fallback: every compute entry point launches a
// gfx950 kernel or returns an error.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/pfe.h"
#include "bates_common.h"
#include "options.h"
#include "pfd.h"

namespace pfe {
hipError_t launch_lyon8_u8(const uint8_t* prof, int64_t ps, int lp, const uint8_t* dm,
                           int64_t ds, int ld, int64_t n, double* out, hipStream_t st,
                           const Options& o);
hipError_t launch_lyon8_f64(const double* prof, int64_t ps, int lp, const double* dm,
                            int64_t ds, int ld, int64_t n, double* out, hipStream_t st,
                            const Options& o);
hipError_t launch_bates22(const pfe_bates_in* in, double* out, uint32_t* status, void* work,
                          size_t work_bytes, hipStream_t st, const Fork* fk, const Options& o);
size_t bates22_workspace_bytes(const pfe_bates_in* in);
hipError_t launch_bates_groups(const pfe_bates_in* in, double* out, uint32_t* status, void* work,
                               size_t work_bytes, hipStream_t st, const Fork* fk,
                               const Options& o, unsigned groups, bool raw_dm);
hipError_t launch_subband3(const pfe_bates_in* in, double* out, uint32_t* status, void* work,
                           hipStream_t st);
const char* subband_shape_error(int nsub, int lsb);
size_t subband_work_bytes(int64_t n, int nsub, int lsb);
}  // namespace pfe

// chunked host path: device/staging slots in flight (H2D of k+1 | kernel k | D2H of k-1)
constexpr int PIPE_SLOTS = 3;
constexpr size_t PIPE_CHUNK_BYTES = 64u << 20;  // input bytes per chunk

struct pfe_handle {
  int device = -1;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  pfe::Fork fork;  // side streams of the 22-score chains (bates_common.h)
  pfe::Options opt;
  // device scratch: staging of the one-shot host paths, the 22-score workspace and the
  // device slots of the chunked host path
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // completion of the last call, on the stream it ran on: a call on another stream first
  // waits for it, so work on the shared scratch never overlaps
  hipEvent_t done = nullptr;
  hipStream_t last = nullptr;
  bool done_recorded = false;
  // chunked host path: copy streams, per-slot events and the pinned staging ring
  hipStream_t h2d = nullptr, d2h = nullptr;
  hipEvent_t ev_in[PIPE_SLOTS] = {}, ev_k[PIPE_SLOTS] = {}, ev_out[PIPE_SLOTS] = {};
  void* pin = nullptr;
  size_t pin_bytes = 0;
  size_t scratch_bytes_peak = 0;  // the largest scratch allocated (growth policy)
  // split PFD pipeline (pfe_pfd_dmprof): two events per part-sum buffer, made on first use
  hipEvent_t pev[4] = {};
  std::string err;
};

static thread_local std::string g_create_err;

static int set_err(pfe_handle* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (h)
    h->err = buf;
  else
    g_create_err = buf;
  return code;
}

#define PFE_HIP(h, expr)                                                                   \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return set_err((h), PFE_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(e_));     \
  } while (0)

// every compute call: bind the device and order after the previous call of this handle
static int call_begin(pfe_handle* h) {
  PFE_HIP(h, hipSetDevice(h->device));
  if (h->done_recorded && h->last != h->stream) PFE_HIP(h, hipStreamWaitEvent(h->stream, h->done, 0));
  return PFE_OK;
}
static int call_end(pfe_handle* h) {
  PFE_HIP(h, hipEventRecord(h->done, h->stream));
  h->done_recorded = true;
  h->last = h->stream;
  return PFE_OK;
}

static int ensure_scratch(pfe_handle* h, size_t bytes) {
  if (bytes <= h->scratch_bytes) return PFE_OK;
  if (h->scratch) {
    // every earlier call's work on the old scratch has finished before it is freed
    if (h->done_recorded) PFE_HIP(h, hipEventSynchronize(h->done));
    PFE_HIP(h, hipStreamSynchronize(h->stream));
    PFE_HIP(h, hipFree(h->scratch));
    h->scratch = nullptr;
    h->scratch_bytes = 0;
  }
  // grow geometrically (4x the previous peak, below 1 GiB): a run whose batches grow (a
  // ramped start) reallocates (device-wide synchronising free) once or twice, not at every
  // size -- but never beyond twice what this call asked for, so a handle does not keep
  // several GiB for moderate batches
  const size_t old = h->scratch_bytes_peak;
  size_t want = bytes + (bytes >> 3) + 4096;
  size_t geo = old * 4 < ((size_t)1 << 30) ? old * 4 : ((size_t)1 << 30);
  if (geo > 2 * bytes) geo = 2 * bytes;
  if (geo > want) want = geo;
  PFE_HIP(h, hipMalloc(&h->scratch, want));
  h->scratch_bytes_peak = want;
  h->scratch_bytes = want;
  return PFE_OK;
}

static int ensure_pinned(pfe_handle* h, size_t bytes) {
  if (bytes <= h->pin_bytes) return PFE_OK;
  if (h->pin) {
    PFE_HIP(h, hipHostFree(h->pin));
    h->pin = nullptr;
    h->pin_bytes = 0;
  }
  PFE_HIP(h, hipHostMalloc(&h->pin, bytes, hipHostMallocDefault));
  h->pin_bytes = bytes;
  return PFE_OK;
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// host memory the DMA engines can read directly (hipHostMalloc / hipHostRegister)
static bool is_pinned(const void* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

extern "C" {

int pfe_abi_version(void) { return PFE_ABI_VERSION; }

int pfe_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int pfe_create(int device, pfe_handle** out) {
  if (!out) return set_err(nullptr, PFE_EINVAL, "pfe_create: out is NULL");
  *out = nullptr;
  if (device < 0)
    return set_err(nullptr, PFE_ENODEV,
                   "pfe_create: device %d: libpfe has no CPU backend; a gfx950 GPU is required",
                   device);
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return set_err(nullptr, PFE_ENODEV, "pfe_create: no HIP device visible (%s)",
                   hipGetErrorString(e));
  if (device >= n)
    return set_err(nullptr, PFE_ENODEV, "pfe_create: device %d out of range (%d visible)",
                   device, n);
  pfe_handle* h = new (std::nothrow) pfe_handle();
  if (!h) return set_err(nullptr, PFE_EDEVICE, "pfe_create: out of host memory");
  h->device = device;
  if ((e = hipSetDevice(device)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking)) != hipSuccess) {
    delete h;
    return set_err(nullptr, PFE_EDEVICE, "pfe_create: %s", hipGetErrorString(e));
  }
  h->stream = h->own;
  for (int i = 0; i < 2 && e == hipSuccess; ++i)
    e = hipStreamCreateWithFlags(&h->fork.side[i], hipStreamNonBlocking);
  for (int i = 0; i < 3 && e == hipSuccess; ++i)
    e = hipEventCreateWithFlags(&h->fork.ev[i], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->done, hipEventDisableTiming);
  if (e != hipSuccess) {
    pfe_destroy(h);
    return set_err(nullptr, PFE_EDEVICE, "pfe_create: %s", hipGetErrorString(e));
  }
  *out = h;
  return PFE_OK;
}

void pfe_destroy(pfe_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->done_recorded) (void)hipEventSynchronize(h->done);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->h2d) (void)hipStreamSynchronize(h->h2d);
  if (h->d2h) (void)hipStreamSynchronize(h->d2h);
  if (h->scratch) (void)hipFree(h->scratch);
  if (h->pin) (void)hipHostFree(h->pin);
  for (hipStream_t& s : h->fork.side)
    if (s) (void)hipStreamDestroy(s);
  for (hipEvent_t& v : h->fork.ev)
    if (v) (void)hipEventDestroy(v);
  for (hipEvent_t& v : h->pev)
    if (v) (void)hipEventDestroy(v);
  for (int i = 0; i < PIPE_SLOTS; ++i) {
    if (h->ev_in[i]) (void)hipEventDestroy(h->ev_in[i]);
    if (h->ev_k[i]) (void)hipEventDestroy(h->ev_k[i]);
    if (h->ev_out[i]) (void)hipEventDestroy(h->ev_out[i]);
  }
  if (h->h2d) (void)hipStreamDestroy(h->h2d);
  if (h->d2h) (void)hipStreamDestroy(h->d2h);
  if (h->done) (void)hipEventDestroy(h->done);
  if (h->own) (void)hipStreamDestroy(h->own);
  delete h;
}

const char* pfe_last_error(const pfe_handle* h) {
  return h ? h->err.c_str() : g_create_err.c_str();
}

int pfe_set_stream(pfe_handle* h, void* s) {
  if (!h) return PFE_EINVAL;
  h->stream = (hipStream_t)s;  // NULL selects the HIP default (null) stream
  return PFE_OK;
}

int pfe_synchronize(pfe_handle* h) {
  if (!h) return PFE_EINVAL;
  PFE_HIP(h, hipSetDevice(h->device));
  PFE_HIP(h, hipStreamSynchronize(h->stream));
  return PFE_OK;
}

int pfe_set_option(pfe_handle* h, int32_t option, int64_t v) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  pfe::Options& o = h->opt;
  switch (option) {
    case PFE_OPT_SOLVER:
      if (v != PFE_SOLVER_POOLED && v != PFE_SOLVER_BATCHED && v != PFE_SOLVER_WAVE) break;
      o.solver = (int)v;
      return PFE_OK;
    case PFE_OPT_SERIAL:
      if (v != 0 && v != 1) break;
      o.serial = (int)v;
      h->fork.serial = (int)v;
      return PFE_OK;
    case PFE_OPT_HANDOVER:
      if (v != 0 && v != 1) break;
      o.handover = (int)v;
      return PFE_OK;
    case PFE_OPT_GSLOTS:
      if (v < 0 || v > pfe::GLM_FPW) break;
      o.gslots = (int)v;
      return PFE_OK;
    case PFE_OPT_LYON8_BLOCKS:
      if (v < 1 || v > (1 << 24)) break;
      o.lyon8_blocks = (int)v;
      return PFE_OK;
    case PFE_OPT_LYON8_BURST:
      if (v != 1 && v != 2 && v != 4) break;
      o.lyon8_burst = (int)v;
      return PFE_OK;
    case PFE_OPT_PFD_WAVES:
      if (v != 1 && v != 4) break;
      o.pfd_waves = (int)v;
      return PFE_OK;
    case PFE_OPT_LYON8_DM:
      if (v < 0 || v > 2) break;
      o.lyon8_dm = (int)v;
      return PFE_OK;
    case PFE_OPT_PFD_SPLIT:
      if (v != 0 && v != 1) break;
      o.pfd_split = (int)v;
      return PFE_OK;
    case PFE_OPT_LYON8_DM_SPLIT:
      if (v < 0 || v > 2) break;
      o.lyon8_dm_split = (int)v;
      return PFE_OK;
    default:
      return set_err(h, PFE_EINVAL, "pfe_set_option: unknown option %d", option);
  }
  return set_err(h, PFE_EINVAL, "pfe_set_option: value %lld out of range for option %d",
                 (long long)v, option);
}

int pfe_get_option(const pfe_handle* h, int32_t option, int64_t* v) {
  if (!h || !v) return PFE_EINVAL;
  const pfe::Options& o = h->opt;
  switch (option) {
    case PFE_OPT_SOLVER: *v = o.solver; return PFE_OK;
    case PFE_OPT_SERIAL: *v = o.serial; return PFE_OK;
    case PFE_OPT_HANDOVER: *v = o.handover; return PFE_OK;
    case PFE_OPT_GSLOTS: *v = o.gslots; return PFE_OK;
    case PFE_OPT_LYON8_BLOCKS: *v = o.lyon8_blocks; return PFE_OK;
    case PFE_OPT_LYON8_BURST: *v = o.lyon8_burst; return PFE_OK;
    case PFE_OPT_PFD_WAVES: *v = o.pfd_waves; return PFE_OK;
    case PFE_OPT_LYON8_DM: *v = o.lyon8_dm; return PFE_OK;
    case PFE_OPT_PFD_SPLIT: *v = o.pfd_split; return PFE_OK;
    case PFE_OPT_LYON8_DM_SPLIT: *v = o.lyon8_dm_split; return PFE_OK;
    default: return PFE_EINVAL;
  }
}

int pfe_host_alloc(size_t bytes, void** out) {
  if (!out) return PFE_EINVAL;
  *out = nullptr;
  if (bytes == 0) bytes = 1;
  if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return PFE_EDEVICE;
  }
  return PFE_OK;
}

void pfe_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

}  // extern "C"

// ---- 8 Lyon features ------------------------------------------------------------------
template <typename T>
static hipError_t launch_lyon8(const T* prof, int64_t ps, int lp, const T* dm, int64_t ds, int ld,
                               int64_t n, double* out, hipStream_t st, const pfe::Options& o) {
  if constexpr (sizeof(T) == 1)
    return pfe::launch_lyon8_u8((const uint8_t*)prof, ps, lp, (const uint8_t*)dm, ds, ld, n, out,
                                st, o);
  else
    return pfe::launch_lyon8_f64((const double*)prof, ps, lp, (const double*)dm, ds, ld, n, out,
                                 st, o);
}

// rows [r0, r0 + rows) of a strided host array into a dense buffer
template <typename T>
static void pack_rows(T* dst, const T* src, int64_t stride, int len, int64_t r0, int64_t rows) {
  if (stride == len) {
    memcpy(dst, src + r0 * stride, (size_t)rows * len * sizeof(T));
    return;
  }
  for (int64_t r = 0; r < rows; ++r)
    memcpy(dst + r * len, src + (r0 + r) * stride, (size_t)len * sizeof(T));
}

// The host-pointer path, chunked and pipelined: chunk k's rows go host -> HBM on the h2d
// stream while chunk k-1's kernel runs on the handle's stream and chunk k-2's features go
// back on the d2h stream.  Pinned caller buffers (pfe_host_alloc) are DMA'd in place;
// pageable ones are packed into (or unpacked from) the handle's pinned staging ring by the
// calling thread, overlapped with the DMA of the other slots.
template <typename T>
static int lyon8_host(pfe_handle* h, const T* prof, int64_t ps, int32_t lp, const T* dm,
                      int64_t ds, int32_t ld, int64_t n, double* out) {
  const size_t row_in = (size_t)(lp + ld) * sizeof(T);
  int64_t chunk = (int64_t)(PIPE_CHUNK_BYTES / row_in);
  chunk = std::max<int64_t>(1024, chunk & ~(int64_t)63);
  if (chunk > n) chunk = n;
  const size_t pb = align256((size_t)chunk * lp * sizeof(T));
  const size_t db = align256((size_t)chunk * ld * sizeof(T));
  const size_t ob = align256((size_t)chunk * 8 * sizeof(double));
  const size_t slot = pb + db + ob;
  int rc = ensure_scratch(h, PIPE_SLOTS * slot);
  if (rc) return rc;
  const bool pin_p = is_pinned(prof), pin_d = is_pinned(dm), pin_o = is_pinned(out);
  if (!(pin_p && pin_d && pin_o)) {
    rc = ensure_pinned(h, PIPE_SLOTS * slot);
    if (rc) return rc;
  }
  if (!h->h2d) {
    PFE_HIP(h, hipStreamCreateWithFlags(&h->h2d, hipStreamNonBlocking));
    PFE_HIP(h, hipStreamCreateWithFlags(&h->d2h, hipStreamNonBlocking));
    for (int i = 0; i < PIPE_SLOTS; ++i) {
      PFE_HIP(h, hipEventCreateWithFlags(&h->ev_in[i], hipEventDisableTiming));
      PFE_HIP(h, hipEventCreateWithFlags(&h->ev_k[i], hipEventDisableTiming));
      PFE_HIP(h, hipEventCreateWithFlags(&h->ev_out[i], hipEventDisableTiming));
    }
  }
  // the copy streams start after the work already queued on the handle's stream
  PFE_HIP(h, hipEventRecord(h->done, h->stream));
  PFE_HIP(h, hipStreamWaitEvent(h->h2d, h->done, 0));
  PFE_HIP(h, hipStreamWaitEvent(h->d2h, h->done, 0));
  const int64_t K = (n + chunk - 1) / chunk;
  auto rows_of = [&](int64_t k) { return std::min<int64_t>(chunk, n - k * chunk); };
  auto unstage_out = [&](int64_t k) -> int {  // pageable out: staging -> caller, after D2H k
    const int s = (int)(k % PIPE_SLOTS);
    PFE_HIP(h, hipEventSynchronize(h->ev_out[s]));
    if (!pin_o)
      memcpy(out + k * chunk * 8, (char*)h->pin + s * slot + pb + db,
             (size_t)rows_of(k) * 8 * sizeof(double));
    return PFE_OK;
  };
  for (int64_t k = 0; k < K; ++k) {
    const int s = (int)(k % PIPE_SLOTS);
    const int64_t r0 = k * chunk, rows = rows_of(k);
    char* dslot = (char*)h->scratch + s * slot;
    char* hslot = h->pin ? (char*)h->pin + s * slot : nullptr;
    T* dprof = (T*)dslot;
    T* ddm = (T*)(dslot + pb);
    double* dout = (double*)(dslot + pb + db);
    if (k >= PIPE_SLOTS) {
      // slot reuse: chunk k-3's staged output is drained (and with it its H2D and kernel)
      rc = unstage_out(k - PIPE_SLOTS);
      if (rc) return rc;
    }
    if (!pin_p) pack_rows((T*)hslot, prof, ps, lp, r0, rows);
    if (!pin_d) pack_rows((T*)(hslot + pb), dm, ds, ld, r0, rows);
    if (pin_p && ps == lp)
      PFE_HIP(h, hipMemcpyAsync(dprof, prof + r0 * ps, (size_t)rows * lp * sizeof(T),
                                hipMemcpyHostToDevice, h->h2d));
    else if (pin_p)
      PFE_HIP(h, hipMemcpy2DAsync(dprof, lp * sizeof(T), prof + r0 * ps, ps * sizeof(T),
                                  lp * sizeof(T), rows, hipMemcpyHostToDevice, h->h2d));
    else
      PFE_HIP(h, hipMemcpyAsync(dprof, hslot, (size_t)rows * lp * sizeof(T),
                                hipMemcpyHostToDevice, h->h2d));
    if (pin_d && ds == ld)
      PFE_HIP(h, hipMemcpyAsync(ddm, dm + r0 * ds, (size_t)rows * ld * sizeof(T),
                                hipMemcpyHostToDevice, h->h2d));
    else if (pin_d)
      PFE_HIP(h, hipMemcpy2DAsync(ddm, ld * sizeof(T), dm + r0 * ds, ds * sizeof(T),
                                  ld * sizeof(T), rows, hipMemcpyHostToDevice, h->h2d));
    else
      PFE_HIP(h, hipMemcpyAsync(ddm, hslot + pb, (size_t)rows * ld * sizeof(T),
                                hipMemcpyHostToDevice, h->h2d));
    PFE_HIP(h, hipEventRecord(h->ev_in[s], h->h2d));
    PFE_HIP(h, hipStreamWaitEvent(h->stream, h->ev_in[s], 0));
    hipError_t e = launch_lyon8<T>(dprof, lp, lp, ddm, ld, ld, rows, dout, h->stream, h->opt);
    if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "lyon8 launch: %s", hipGetErrorString(e));
    PFE_HIP(h, hipEventRecord(h->ev_k[s], h->stream));
    PFE_HIP(h, hipStreamWaitEvent(h->d2h, h->ev_k[s], 0));
    PFE_HIP(h, hipMemcpyAsync(pin_o ? (void*)(out + r0 * 8) : (void*)(hslot + pb + db), dout,
                              (size_t)rows * 8 * sizeof(double), hipMemcpyDeviceToHost, h->d2h));
    PFE_HIP(h, hipEventRecord(h->ev_out[s], h->d2h));
  }
  for (int64_t k = std::max<int64_t>(0, K - PIPE_SLOTS); k < K; ++k) {
    rc = unstage_out(k);
    if (rc) return rc;
  }
  return PFE_OK;
}

template <typename T>
static int lyon8_impl(pfe_handle* h, const T* prof, int64_t ps, int32_t lp, const T* dm,
                      int64_t ds, int32_t ld, int64_t n, double* out, uint32_t* status,
                      uint32_t flags, bool is_u8) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (n < 0) return set_err(h, PFE_EINVAL, "lyon8: n=%lld < 0", (long long)n);
  if (lp < 1 || ld < 1) return set_err(h, PFE_EINVAL, "lyon8: lp=%d ld=%d must be >= 1", lp, ld);
  if (ps < lp || ds < ld)
    return set_err(h, PFE_EINVAL, "lyon8: strides (%lld,%lld) shorter than rows (%d,%d)",
                   (long long)ps, (long long)ds, lp, ld);
  if (n == 0) return PFE_OK;
  if (!prof || !dm || !out) return set_err(h, PFE_EINVAL, "lyon8: null buffer");
  if (!is_u8 && (lp > (1 << 30) || ld > (1 << 30)))
    return set_err(h, PFE_EINVAL, "lyon8: row too long");
  if (is_u8 && (lp >= (1 << 24) || ld >= (1 << 24)))
    return set_err(h, PFE_EINVAL, "lyon8_u8: rows must be shorter than 2^24 bins");
  int rc = call_begin(h);
  if (rc) return rc;
  if (flags & PFE_FLAG_DEVICE_PTRS) {
    hipError_t e = launch_lyon8<T>(prof, ps, lp, dm, ds, ld, n, out, h->stream, h->opt);
    if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "lyon8 launch: %s", hipGetErrorString(e));
    if (status) PFE_HIP(h, hipMemsetAsync(status, 0, (size_t)n * sizeof(uint32_t), h->stream));
    return call_end(h);
  }
  rc = lyon8_host<T>(h, prof, ps, lp, dm, ds, ld, n, out);
  if (rc) return rc;
  if (status) memset(status, 0, (size_t)n * sizeof(uint32_t));
  return call_end(h);
}

extern "C" {

int pfe_lyon8_u8(pfe_handle* h, const uint8_t* prof, int64_t ps, int32_t lp, const uint8_t* dm,
                 int64_t ds, int32_t ld, int64_t n, double* out, uint32_t* status,
                 uint32_t flags) {
  return lyon8_impl<uint8_t>(h, prof, ps, lp, dm, ds, ld, n, out, status, flags, true);
}

int pfe_lyon8_f64(pfe_handle* h, const double* prof, int64_t ps, int32_t lp, const double* dm,
                  int64_t ds, int32_t ld, int64_t n, double* out, uint32_t* status,
                  uint32_t flags) {
  return lyon8_impl<double>(h, prof, ps, lp, dm, ds, ld, n, out, status, flags, false);
}

}  // extern "C"

// ---- 22 Bates scores / sub-band scores -------------------------------------------------
static int check_bates_in(pfe_handle* h, const pfe_bates_in* in, const char* fn, bool need_dm) {
  if (!in->prof || !in->sub || !in->scal || (need_dm && !in->dmcurve))
    return set_err(h, PFE_EINVAL, "%s: null input array", fn);
  // the 22-score chain's profile kernels take 8-1024 bins; the sub-band scores alone only
  // compare the profile with the sub-bands (any nBins the any-shape kernel holds)
  if (need_dm ? (in->lp < 8 || in->lp > 1024) : (in->lp < 1 || in->lp > 16384))
    return set_err(h, PFE_EINVAL, "%s: lp=%d outside [%d,%d]", fn, in->lp, need_dm ? 8 : 1,
                   need_dm ? 1024 : 16384);
  // pfe_subband3 computes nothing else, so an unsupported sub-band shape fails the call; in
  // pfe_bates22 it only fails the rows' sub-band group (PFE_ST_UNSUPPORTED per row), within
  // the per-candidate bound of 2^24 sub-band bytes that pfe_bates22 itself checks (pfe.h
  // PFE_ST_UNSUPPORTED)
  if (!need_dm) {
    if (const char* why = pfe::subband_shape_error(in->nsub, in->lsb))
      return set_err(h, PFE_EINVAL, "%s: sub-band shape %dx%d: %s", fn, in->nsub, in->lsb, why);
  } else if (in->nsub < 1 || in->lsb < 1 || (int64_t)in->nsub * in->lsb > (1 << 24)) {
    return set_err(h, PFE_EINVAL, "%s: sub-band shape %dx%d", fn, in->nsub, in->lsb);
  }
  if (need_dm && (in->ndm < 3 || in->ndm > 1024))
    return set_err(h, PFE_EINVAL, "%s: ndm=%d outside [3,1024]", fn, in->ndm);
  return PFE_OK;
}

// one-shot staging of a host-pointer batch: inputs -> scratch, then `nout` doubles and a
// status word per row of output space
static int stage_bates(pfe_handle* h, const pfe_bates_in* in, pfe_bates_in& din, int nout,
                       bool with_dm, size_t work, double*& dout, uint32_t*& dstat, size_t& off) {
  const int64_t n = in->n;
  hipStream_t st = h->stream;
  const size_t pb = align256((size_t)n * in->lp);
  const size_t sb = align256((size_t)n * in->nsub * in->lsb);
  const size_t db = with_dm ? align256((size_t)n * in->ndm * sizeof(double)) : 0;
  const size_t cb = align256((size_t)n * PFE_NSCAL * sizeof(double));
  const size_t ob = align256((size_t)n * nout * sizeof(double));
  const size_t tb = align256((size_t)n * sizeof(uint32_t));
  int rc = ensure_scratch(h, pb + sb + db + cb + ob + tb + work);
  if (rc) return rc;
  char* base = (char*)h->scratch;
  PFE_HIP(h, hipMemcpyAsync(base, in->prof, (size_t)n * in->lp, hipMemcpyHostToDevice, st));
  din.prof = (const uint8_t*)base;
  off = pb;
  PFE_HIP(h, hipMemcpyAsync(base + off, in->sub, (size_t)n * in->nsub * in->lsb,
                            hipMemcpyHostToDevice, st));
  din.sub = (const uint8_t*)(base + off);
  off += sb;
  if (with_dm) {
    PFE_HIP(h, hipMemcpyAsync(base + off, in->dmcurve, (size_t)n * in->ndm * sizeof(double),
                              hipMemcpyHostToDevice, st));
    din.dmcurve = (const double*)(base + off);
    off += db;
  }
  PFE_HIP(h, hipMemcpyAsync(base + off, in->scal, (size_t)n * PFE_NSCAL * sizeof(double),
                            hipMemcpyHostToDevice, st));
  din.scal = (const double*)(base + off);
  off += cb;
  dout = (double*)(base + off);
  off += ob;
  dstat = (uint32_t*)(base + off);
  off += tb;
  return PFE_OK;
}

extern "C" {

int pfe_bates22(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                uint32_t flags) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (!in || !out || !status) return set_err(h, PFE_EINVAL, "bates22: null argument");
  const int64_t n = in->n;
  if (n < 0) return set_err(h, PFE_EINVAL, "bates22: n < 0");
  if (n == 0) return PFE_OK;
  int rc = check_bates_in(h, in, "bates22", true);
  if (rc) return rc;
  rc = call_begin(h);
  if (rc) return rc;
  hipStream_t st = h->stream;
  pfe_bates_in din = *in;
  double* dout = out;
  uint32_t* dstat = status;
  size_t off = 0;
  const size_t work = pfe::bates22_workspace_bytes(in);
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    rc = stage_bates(h, in, din, 22, true, work, dout, dstat, off);
  } else {
    rc = ensure_scratch(h, work);
  }
  if (rc) return rc;
  hipError_t e = pfe::launch_bates22(&din, dout, dstat, (char*)h->scratch + off, work, st,
                                     &h->fork, h->opt);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "bates22 launch: %s", hipGetErrorString(e));
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    PFE_HIP(h, hipMemcpyAsync(out, dout, (size_t)n * 22 * sizeof(double), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipMemcpyAsync(status, dstat, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return call_end(h);
}

int pfe_subband3(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                 uint32_t flags) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (!in || !out || !status) return set_err(h, PFE_EINVAL, "subband3: null argument");
  const int64_t n = in->n;
  if (n < 0) return set_err(h, PFE_EINVAL, "subband3: n < 0");
  if (n == 0) return PFE_OK;
  int rc = check_bates_in(h, in, "subband3", false);
  if (rc) return rc;
  rc = call_begin(h);
  if (rc) return rc;
  hipStream_t st = h->stream;
  pfe_bates_in din = *in;
  double* dout = out;
  uint32_t* dstat = status;
  size_t off = 0;
  const size_t work = pfe::subband_work_bytes(n, in->nsub, in->lsb);
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    rc = stage_bates(h, in, din, 3, false, work ? work + 256 : 0, dout, dstat, off);
  } else if (work) {
    rc = ensure_scratch(h, work + 256);
  }
  if (rc) return rc;
  void* wp = work ? (void*)(((uintptr_t)h->scratch + off + 255) & ~(uintptr_t)255) : nullptr;
  hipError_t e = pfe::launch_subband3(&din, dout, dstat, wp, st);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "subband3 launch: %s", hipGetErrorString(e));
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    PFE_HIP(h, hipMemcpyAsync(out, dout, (size_t)n * 3 * sizeof(double), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipMemcpyAsync(status, dstat, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return call_end(h);
}

}  // extern "C"

// ---- one score group of the chain (ProfileOperationsInterface.py:69-130) ----------------
// columns [c0, c0 + k) of the 22-score vector -> dst (n x k)
__global__ void k_take_cols(const double* src, int c0, int k, int64_t n, double* dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * k) dst[i] = src[(i / k) * 22 + c0 + i % k];
}

// getCandidateParameters: (period, snr, dm, width) of each candidate, unfiltered
__global__ void k_params4(const double* scal, int64_t n, double* out, uint32_t* status) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* sc = scal + i * PFE_NSCAL;
  out[i * 4 + 0] = sc[PFE_SCAL_PERIOD_MS];
  out[i * 4 + 1] = sc[PFE_SCAL_SNR];
  out[i * 4 + 2] = sc[PFE_SCAL_DM];
  out[i * 4 + 3] = sc[PFE_SCAL_WIDTH];
  status[i] = 0;
}

// groups: pfe::BG_SINE (cols 0-3) / BG_GAUSS (4-10) / BG_DM (15-18, raw shift)
static int bates_group_call(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                            uint32_t flags, const char* fn, unsigned groups, int c0, int k) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (!in || !out || !status) return set_err(h, PFE_EINVAL, "%s: null argument", fn);
  const int64_t n = in->n;
  if (n < 0) return set_err(h, PFE_EINVAL, "%s: n < 0", fn);
  if (n == 0) return PFE_OK;
  const bool dm = groups == pfe::BG_DM;
  if (!in->scal || (dm ? !in->dmcurve : !in->prof))
    return set_err(h, PFE_EINVAL, "%s: null input array", fn);
  if (!dm && (in->lp < 8 || in->lp > 1024))
    return set_err(h, PFE_EINVAL, "%s: lp=%d outside [8,1024]", fn, in->lp);
  if (dm && (in->ndm < 3 || in->ndm > 1024))
    return set_err(h, PFE_EINVAL, "%s: ndm=%d outside [3,1024]", fn, in->ndm);
  int rc = call_begin(h);
  if (rc) return rc;
  hipStream_t st = h->stream;
  // only the arrays the group reads; no sub-band work
  pfe_bates_in g = *in;
  g.sub = nullptr;
  g.nsub = g.lsb = 0;
  if (dm) {
    g.prof = nullptr;
    g.lp = 0;
  } else {
    g.dmcurve = nullptr;
    g.ndm = 0;
  }
  const bool host = !(flags & PFE_FLAG_DEVICE_PTRS);
  const size_t work = pfe::bates22_workspace_bytes(&g);
  const size_t pb = host && !dm ? align256((size_t)n * g.lp) : 0;
  const size_t db = host && dm ? align256((size_t)n * g.ndm * sizeof(double)) : 0;
  const size_t cb = host ? align256((size_t)n * PFE_NSCAL * sizeof(double)) : 0;
  const size_t ob = align256((size_t)n * 22 * sizeof(double));
  const size_t kb = host ? align256((size_t)n * k * sizeof(double)) : 0;
  const size_t tb = host ? align256((size_t)n * sizeof(uint32_t)) : 0;
  rc = ensure_scratch(h, pb + db + cb + ob + kb + tb + work + 256);
  if (rc) return rc;
  char* base = (char*)(((uintptr_t)h->scratch + 255) & ~(uintptr_t)255);
  pfe_bates_in din = g;
  size_t off = 0;
  if (host) {
    if (dm) {
      PFE_HIP(h, hipMemcpyAsync(base, in->dmcurve, (size_t)n * g.ndm * sizeof(double),
                                hipMemcpyHostToDevice, st));
      din.dmcurve = (const double*)base;
    } else {
      PFE_HIP(h, hipMemcpyAsync(base, in->prof, (size_t)n * g.lp, hipMemcpyHostToDevice, st));
      din.prof = (const uint8_t*)base;
    }
    off = pb + db;
    PFE_HIP(h, hipMemcpyAsync(base + off, in->scal, (size_t)n * PFE_NSCAL * sizeof(double),
                              hipMemcpyHostToDevice, st));
    din.scal = (const double*)(base + off);
    off += cb;
  }
  double* d22 = (double*)(base + off);
  off += ob;
  double* dk = host ? (double*)(base + off) : out;
  off += kb;
  uint32_t* dst = host ? (uint32_t*)(base + off) : status;
  off += tb;
  hipError_t e = pfe::launch_bates_groups(&din, d22, dst, base + off, work, st, &h->fork, h->opt,
                                          groups, dm);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "%s launch: %s", fn, hipGetErrorString(e));
  hipLaunchKernelGGL(k_take_cols, dim3((unsigned)((n * k + 255) / 256)), dim3(256), 0, st, d22,
                     c0, k, n, dk);
  PFE_HIP(h, hipGetLastError());
  if (host) {
    PFE_HIP(h, hipMemcpyAsync(out, dk, (size_t)n * k * sizeof(double), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipMemcpyAsync(status, dst, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return call_end(h);
}

extern "C" {

int pfe_sinusoid4(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                  uint32_t flags) {
  return bates_group_call(h, in, out, status, flags, "sinusoid4", pfe::BG_SINE, 0, 4);
}

int pfe_gauss7(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
               uint32_t flags) {
  return bates_group_call(h, in, out, status, flags, "gauss7", pfe::BG_GAUSS, 4, 7);
}

int pfe_dmfit4(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
               uint32_t flags) {
  return bates_group_call(h, in, out, status, flags, "dmfit4", pfe::BG_DM, 15, 4);
}

int pfe_params4(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                uint32_t flags) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (!in || !out || !status || (in->n > 0 && !in->scal))
    return set_err(h, PFE_EINVAL, "params4: null argument");
  const int64_t n = in->n;
  if (n < 0) return set_err(h, PFE_EINVAL, "params4: n < 0");
  if (n == 0) return PFE_OK;
  int rc = call_begin(h);
  if (rc) return rc;
  hipStream_t st = h->stream;
  if (flags & PFE_FLAG_DEVICE_PTRS) {
    hipLaunchKernelGGL(k_params4, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in->scal,
                       n, out, status);
    PFE_HIP(h, hipGetLastError());
    return call_end(h);
  }
  const size_t cb = align256((size_t)n * PFE_NSCAL * sizeof(double));
  const size_t ob = align256((size_t)n * 4 * sizeof(double));
  rc = ensure_scratch(h, cb + ob + (size_t)n * sizeof(uint32_t));
  if (rc) return rc;
  char* base = (char*)h->scratch;
  PFE_HIP(h, hipMemcpyAsync(base, in->scal, (size_t)n * PFE_NSCAL * sizeof(double),
                            hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_params4, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (const double*)base, n, (double*)(base + cb), (uint32_t*)(base + cb + ob));
  PFE_HIP(h, hipGetLastError());
  PFE_HIP(h, hipMemcpyAsync(out, base + cb, (size_t)n * 4 * sizeof(double), hipMemcpyDeviceToHost, st));
  PFE_HIP(h, hipMemcpyAsync(status, base + cb + ob, (size_t)n * sizeof(uint32_t),
                            hipMemcpyDeviceToHost, st));
  PFE_HIP(h, hipStreamSynchronize(st));
  return call_end(h);
}

// ---- PFD -------------------------------------------------------------------------------
int pfe_pfd_dmprof(pfe_handle* h, const pfe_pfd_in* in, double* profile, float* chis,
                   double* lyon8, uint32_t* status, uint32_t flags) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (!in || !status) return set_err(h, PFE_EINVAL, "pfd_dmprof: null argument");
  const int64_t n = in->n;
  if (n < 0) return set_err(h, PFE_EINVAL, "pfd_dmprof: n < 0");
  if (n == 0) return PFE_OK;
  if (!in->profs || !in->subfreqs || !in->scal)
    return set_err(h, PFE_EINVAL, "pfd_dmprof: null input array");
  if (in->npart < 1 || in->nsub < 1 || in->proflen < 2)
    return set_err(h, PFE_EINVAL, "pfd_dmprof: shape %dx%dx%d", in->npart, in->nsub, in->proflen);
  if (pfe::pfd_lds_bytes(in->nsub, in->proflen) > 160 * 1024)
    return set_err(h, PFE_EINVAL, "pfd_dmprof: nsub*proflen=%d exceeds the LDS-resident limit",
                   in->nsub * in->proflen);
  int rc = call_begin(h);
  if (rc) return rc;
  hipStream_t st = h->stream;
  pfe::PfdArgs a;
  a.npart = in->npart;
  a.nsub = in->nsub;
  a.L = in->proflen;
  a.n = n;
  a.waves = h->opt.pfd_waves;
  const size_t np = (size_t)n * in->npart * in->nsub * in->proflen;
  // split pipeline: two buffers of part sums, chunks of up to 4096 folds
  // (2 x 4096 x nsub x L doubles: 268 MB at 32 x 128)
  const bool split = h->opt.pfd_split && h->fork.side[0] && pfe::pfd_split_ok(a);
  const int64_t chunk = n < 4096 ? n : 4096;
  const size_t wsb = split ? align256(2 * (size_t)chunk * in->nsub * in->proflen * sizeof(double)) : 0;
  size_t wsoff = 0;
  if (split) {
    for (hipEvent_t& v : h->pev)
      if (!v) PFE_HIP(h, hipEventCreateWithFlags(&v, hipEventDisableTiming));
  }
  if (flags & PFE_FLAG_DEVICE_PTRS) {
    if (split) {
      rc = ensure_scratch(h, wsb);
      if (rc) return rc;
    }
    a.profs = in->profs;
    a.subfreqs = in->subfreqs;
    a.scal = in->scal;
    a.profile = profile;
    a.chis = chis;
    a.lyon8 = lyon8;
    a.status = status;
  } else {
    const size_t pb = align256(np * sizeof(double));
    const size_t fb = align256((size_t)n * in->nsub * sizeof(double));
    const size_t cb = align256((size_t)n * PFE_PFD_NSCAL * sizeof(double));
    const size_t ob = profile ? align256((size_t)n * in->proflen * sizeof(double)) : 0;
    const size_t xb = chis ? align256((size_t)n * PFE_PFD_NDM * sizeof(float)) : 0;
    const size_t lb = lyon8 ? align256((size_t)n * 8 * sizeof(double)) : 0;
    const size_t tb = align256((size_t)n * sizeof(uint32_t));
    rc = ensure_scratch(h, pb + fb + cb + ob + xb + lb + tb + wsb);
    if (rc) return rc;
    wsoff = pb + fb + cb + ob + xb + lb + tb;
    char* base = (char*)h->scratch;
    size_t off = 0;
    PFE_HIP(h, hipMemcpyAsync(base, in->profs, np * sizeof(double), hipMemcpyHostToDevice, st));
    a.profs = (const double*)base;
    off += pb;
    PFE_HIP(h, hipMemcpyAsync(base + off, in->subfreqs, (size_t)n * in->nsub * sizeof(double),
                              hipMemcpyHostToDevice, st));
    a.subfreqs = (const double*)(base + off);
    off += fb;
    PFE_HIP(h, hipMemcpyAsync(base + off, in->scal, (size_t)n * PFE_PFD_NSCAL * sizeof(double),
                              hipMemcpyHostToDevice, st));
    a.scal = (const double*)(base + off);
    off += cb;
    a.profile = profile ? (double*)(base + off) : nullptr;
    off += ob;
    a.chis = chis ? (float*)(base + off) : nullptr;
    off += xb;
    a.lyon8 = lyon8 ? (double*)(base + off) : nullptr;
    off += lb;
    a.status = (uint32_t*)(base + off);
  }
  hipError_t e = split ? pfe::launch_pfd_dmprof_split(a, st, h->fork.side[0],
                                                      (double*)((char*)h->scratch + wsoff), chunk,
                                                      h->pev)
                       : pfe::launch_pfd_dmprof(a, st);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "pfd_dmprof launch: %s", hipGetErrorString(e));
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    if (profile)
      PFE_HIP(h, hipMemcpyAsync(profile, a.profile, (size_t)n * in->proflen * sizeof(double),
                                hipMemcpyDeviceToHost, st));
    if (chis)
      PFE_HIP(h, hipMemcpyAsync(chis, a.chis, (size_t)n * PFE_PFD_NDM * sizeof(float),
                                hipMemcpyDeviceToHost, st));
    if (lyon8)
      PFE_HIP(h, hipMemcpyAsync(lyon8, a.lyon8, (size_t)n * 8 * sizeof(double),
                                hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipMemcpyAsync(status, a.status, (size_t)n * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return call_end(h);
}

int pfe_pfd_bates22(pfe_handle* h, const pfe_pfd_in* in, double* out, uint32_t* status,
                    uint32_t flags) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (!in || !out || !status) return set_err(h, PFE_EINVAL, "pfd_bates22: null argument");
  const int64_t n = in->n;
  if (n < 0) return set_err(h, PFE_EINVAL, "pfd_bates22: n < 0");
  if (n == 0) return PFE_OK;
  if (!in->profs || !in->subfreqs || !in->scal)
    return set_err(h, PFE_EINVAL, "pfd_bates22: null input array");
  if (in->npart < 1 || in->nsub < 2 || in->proflen < 8 || in->proflen > 1024)
    return set_err(h, PFE_EINVAL, "pfd_bates22: shape %dx%dx%d unsupported", in->npart, in->nsub,
                   in->proflen);
  if (pfe::pfd_lds_bytes(in->nsub, in->proflen) > 160 * 1024)
    return set_err(h, PFE_EINVAL, "pfd_bates22: nsub*proflen=%d exceeds the LDS-resident limit",
                   in->nsub * in->proflen);
  int rc = call_begin(h);
  if (rc) return rc;
  hipStream_t st = h->stream;
  pfe::PfdArgs a;
  a.npart = in->npart;
  a.nsub = in->nsub;
  a.L = in->proflen;
  a.n = n;
  a.waves = h->opt.pfd_waves;
  const size_t work = pfe::pfd22_workspace_bytes(n, in->proflen);
  const size_t np = (size_t)n * in->npart * in->nsub * in->proflen;
  double* dout = out;
  uint32_t* dstat = status;
  size_t off = 0;
  if (flags & PFE_FLAG_DEVICE_PTRS) {
    rc = ensure_scratch(h, work);
    if (rc) return rc;
    a.profs = in->profs;
    a.subfreqs = in->subfreqs;
    a.scal = in->scal;
  } else {
    const size_t pb = align256(np * sizeof(double));
    const size_t fb = align256((size_t)n * in->nsub * sizeof(double));
    const size_t cb = align256((size_t)n * PFE_PFD_NSCAL * sizeof(double));
    const size_t ob = align256((size_t)n * 22 * sizeof(double));
    const size_t tb = align256((size_t)n * sizeof(uint32_t));
    rc = ensure_scratch(h, pb + fb + cb + ob + tb + work);
    if (rc) return rc;
    char* base = (char*)h->scratch;
    PFE_HIP(h, hipMemcpyAsync(base, in->profs, np * sizeof(double), hipMemcpyHostToDevice, st));
    a.profs = (const double*)base;
    off += pb;
    PFE_HIP(h, hipMemcpyAsync(base + off, in->subfreqs, (size_t)n * in->nsub * sizeof(double),
                              hipMemcpyHostToDevice, st));
    a.subfreqs = (const double*)(base + off);
    off += fb;
    PFE_HIP(h, hipMemcpyAsync(base + off, in->scal, (size_t)n * PFE_PFD_NSCAL * sizeof(double),
                              hipMemcpyHostToDevice, st));
    a.scal = (const double*)(base + off);
    off += cb;
    dout = (double*)(base + off);
    off += ob;
    dstat = (uint32_t*)(base + off);
    off += tb;
  }
  hipError_t e = pfe::launch_pfd22(a, dout, dstat, (char*)h->scratch + off, work, st, &h->fork,
                                   h->opt);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "pfd_bates22 launch: %s", hipGetErrorString(e));
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    PFE_HIP(h, hipMemcpyAsync(out, dout, (size_t)n * 22 * sizeof(double), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipMemcpyAsync(status, dstat, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return call_end(h);
}

}  // extern "C"

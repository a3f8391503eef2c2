// capi.hip — extern "C" boundary of libpfe.so (declared in include/pfe.h).
//
// Owns: the per-handle HIP stream, device scratch used to stage host buffers, and the
// argument validation that mirrors the reference's failure behaviour.  No CPU fallback:
// every compute entry point launches a gfx950 kernel or returns an error.

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/pfe.h"
#include "bates_common.h"
#include "pfd.h"

namespace pfe {
hipError_t launch_lyon8_u8(const uint8_t* prof, int64_t ps, int lp, const uint8_t* dm,
                           int64_t ds, int ld, int64_t n, double* out, hipStream_t st);
hipError_t launch_lyon8_f64(const double* prof, int64_t ps, int lp, const double* dm,
                            int64_t ds, int ld, int64_t n, double* out, hipStream_t st);
hipError_t launch_bates22(const pfe_bates_in* in, double* out, uint32_t* status, void* work,
                          size_t work_bytes, hipStream_t st, const Fork* fk);
size_t bates22_workspace_bytes(const pfe_bates_in* in);
}  // namespace pfe

struct pfe_handle {
  int device = -1;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  pfe::Fork fork;  // side streams of the 22-score chains (bates_common.h)
  // staging scratch (device)
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
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

static int ensure_scratch(pfe_handle* h, size_t bytes) {
  if (bytes <= h->scratch_bytes) return PFE_OK;
  if (h->scratch) {
    PFE_HIP(h, hipStreamSynchronize(h->stream));
    PFE_HIP(h, hipFree(h->scratch));
    h->scratch = nullptr;
    h->scratch_bytes = 0;
  }
  size_t want = bytes + (bytes >> 3) + 4096;
  PFE_HIP(h, hipMalloc(&h->scratch, want));
  h->scratch_bytes = want;
  return PFE_OK;
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

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
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->scratch) (void)hipFree(h->scratch);
  for (hipStream_t& s : h->fork.side)
    if (s) (void)hipStreamDestroy(s);
  for (hipEvent_t& v : h->fork.ev)
    if (v) (void)hipEventDestroy(v);
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

}  // extern "C"

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
  PFE_HIP(h, hipSetDevice(h->device));
  hipStream_t st = h->stream;
  const T* dprof = prof;
  const T* ddm = dm;
  double* dout = out;
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    // stage dense copies of the rows (row strides collapse to lengths)
    const size_t pb = align256((size_t)n * lp * sizeof(T));
    const size_t db = align256((size_t)n * ld * sizeof(T));
    const size_t ob = align256((size_t)n * 8 * sizeof(double));
    int rc = ensure_scratch(h, pb + db + ob);
    if (rc) return rc;
    char* base = (char*)h->scratch;
    PFE_HIP(h, hipMemcpy2DAsync(base, lp * sizeof(T), prof, ps * sizeof(T), lp * sizeof(T), n,
                                hipMemcpyHostToDevice, st));
    PFE_HIP(h, hipMemcpy2DAsync(base + pb, ld * sizeof(T), dm, ds * sizeof(T), ld * sizeof(T), n,
                                hipMemcpyHostToDevice, st));
    dprof = (const T*)base;
    ddm = (const T*)(base + pb);
    dout = (double*)(base + pb + db);
    ps = lp;
    ds = ld;
  }
  hipError_t e;
  if constexpr (sizeof(T) == 1)
    e = pfe::launch_lyon8_u8((const uint8_t*)dprof, ps, lp, (const uint8_t*)ddm, ds, ld, n,
                             dout, st);
  else
    e = pfe::launch_lyon8_f64((const double*)dprof, ps, lp, (const double*)ddm, ds, ld, n,
                              dout, st);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "lyon8 launch: %s", hipGetErrorString(e));
  if (status) {
    if (flags & PFE_FLAG_DEVICE_PTRS)
      PFE_HIP(h, hipMemsetAsync(status, 0, (size_t)n * sizeof(uint32_t), st));
    else
      memset(status, 0, (size_t)n * sizeof(uint32_t));
  }
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    PFE_HIP(h, hipMemcpyAsync(out, dout, (size_t)n * 8 * sizeof(double), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return PFE_OK;
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

int pfe_bates22(pfe_handle* h, const pfe_bates_in* in, double* out, uint32_t* status,
                uint32_t flags) {
  if (!h) return PFE_EINVAL;
  h->err.clear();
  if (!in || !out || !status) return set_err(h, PFE_EINVAL, "bates22: null argument");
  const int64_t n = in->n;
  if (n < 0) return set_err(h, PFE_EINVAL, "bates22: n < 0");
  if (n == 0) return PFE_OK;
  if (!in->prof || !in->sub || !in->dmcurve || !in->scal)
    return set_err(h, PFE_EINVAL, "bates22: null input array");
  if (in->lp < 8 || in->lp > 1024)
    return set_err(h, PFE_EINVAL, "bates22: lp=%d outside [8,1024]", in->lp);
  if (in->nsub < 2 || in->nsub > 64 || in->lsb < 1 || in->lsb > 1024)
    return set_err(h, PFE_EINVAL, "bates22: sub-band shape %dx%d unsupported", in->nsub, in->lsb);
  if (in->ndm < 3 || in->ndm > 1024)
    return set_err(h, PFE_EINVAL, "bates22: ndm=%d outside [3,1024]", in->ndm);
  PFE_HIP(h, hipSetDevice(h->device));
  hipStream_t st = h->stream;
  pfe_bates_in din = *in;
  double* dout = out;
  uint32_t* dstat = status;
  size_t off = 0;
  const size_t work = pfe::bates22_workspace_bytes(in);
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    const size_t pb = align256((size_t)n * in->lp);
    const size_t sb = align256((size_t)n * in->nsub * in->lsb);
    const size_t db = align256((size_t)n * in->ndm * sizeof(double));
    const size_t cb = align256((size_t)n * PFE_NSCAL * sizeof(double));
    const size_t ob = align256((size_t)n * 22 * sizeof(double));
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
    PFE_HIP(h, hipMemcpyAsync(base + off, in->dmcurve, (size_t)n * in->ndm * sizeof(double),
                              hipMemcpyHostToDevice, st));
    din.dmcurve = (const double*)(base + off);
    off += db;
    PFE_HIP(h, hipMemcpyAsync(base + off, in->scal, (size_t)n * PFE_NSCAL * sizeof(double),
                              hipMemcpyHostToDevice, st));
    din.scal = (const double*)(base + off);
    off += cb;
    dout = (double*)(base + off);
    off += ob;
    dstat = (uint32_t*)(base + off);
    off += tb;
  } else {
    int rc = ensure_scratch(h, work);
    if (rc) return rc;
  }
  hipError_t e = pfe::launch_bates22(&din, dout, dstat, (char*)h->scratch + off, work, st, &h->fork);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "bates22 launch: %s", hipGetErrorString(e));
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    PFE_HIP(h, hipMemcpyAsync(out, dout, (size_t)n * 22 * sizeof(double), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipMemcpyAsync(status, dstat, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return PFE_OK;
}

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
  PFE_HIP(h, hipSetDevice(h->device));
  hipStream_t st = h->stream;
  pfe::PfdArgs a;
  a.npart = in->npart;
  a.nsub = in->nsub;
  a.L = in->proflen;
  a.n = n;
  const size_t np = (size_t)n * in->npart * in->nsub * in->proflen;
  if (flags & PFE_FLAG_DEVICE_PTRS) {
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
    int rc = ensure_scratch(h, pb + fb + cb + ob + xb + lb + tb);
    if (rc) return rc;
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
  hipError_t e = pfe::launch_pfd_dmprof(a, st);
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
  return PFE_OK;
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
  PFE_HIP(h, hipSetDevice(h->device));
  hipStream_t st = h->stream;
  pfe::PfdArgs a;
  a.npart = in->npart;
  a.nsub = in->nsub;
  a.L = in->proflen;
  a.n = n;
  const size_t work = pfe::pfd22_workspace_bytes(n, in->proflen);
  const size_t np = (size_t)n * in->npart * in->nsub * in->proflen;
  double* dout = out;
  uint32_t* dstat = status;
  size_t off = 0;
  if (flags & PFE_FLAG_DEVICE_PTRS) {
    int rc = ensure_scratch(h, work);
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
    int rc = ensure_scratch(h, pb + fb + cb + ob + tb + work);
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
  hipError_t e = pfe::launch_pfd22(a, dout, dstat, (char*)h->scratch + off, work, st, &h->fork);
  if (e != hipSuccess) return set_err(h, PFE_EDEVICE, "pfd_bates22 launch: %s", hipGetErrorString(e));
  if (!(flags & PFE_FLAG_DEVICE_PTRS)) {
    PFE_HIP(h, hipMemcpyAsync(out, dout, (size_t)n * 22 * sizeof(double), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipMemcpyAsync(status, dstat, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PFE_HIP(h, hipStreamSynchronize(st));
  }
  return PFE_OK;
}

}  // extern "C"

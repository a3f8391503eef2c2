// phcx_io.cpp — native PHCX / SUPERB-PHCX reader and batch packer (include/pfe_io.h).
//
// Host code.  One file = gzip (HTRU) or plain (SUPERB) XML; only the leaf elements the
// scores read are extracted, by a single forward scan of the document:
//   Profile, DataBlock, SubBands (nBins, nSub), DmIndex, BaryPeriod, Snr, Dm, Width
// and the k-th occurrence of a tag in document order is what minidom's
// getElementsByTagName(tag)[k] returns (PHCXOperations.py:81-383, PHCXFile.py:144-186).
// Element text follows the XML rules the reference's parser applies (end-of-line
// normalisation, the five predefined entities and character references).  Anything beyond
// that (comments / CDATA / child elements inside a leaf, non-ASCII text, unusual number
// spellings) is reported as a per-file status so the host can use its Python parser for
// that file instead of guessing.
#include <dlfcn.h>
#include <emmintrin.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <charconv>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pfe.h"
#include "../../include/pfe_io.h"

namespace {

enum Tag { T_PROFILE, T_DATABLOCK, T_SUBBANDS, T_DMINDEX, T_BARY, T_SNR, T_DM, T_WIDTH, NTAGS };
const char* const kTagNames[NTAGS] = {"Profile", "DataBlock", "SubBands", "DmIndex",
                                      "BaryPeriod", "Snr", "Dm", "Width"};

struct Elem {
  size_t tb = 0, te = 0;  // raw text range [tb, te) in the document
  bool has_text = false;  // ElementTree's .text is None for empty elements
  bool complex = false;   // text interrupted by a comment / CDATA / child element
  size_t ab = 0, ae = 0;  // raw attribute range
};

struct Parsed {
  pfe_phcx_info info{};
  std::vector<uint8_t> profile, lyon_dm, sub, fit;
  std::vector<double> dmc;
};

// Per-thread buffers: the documents are hundreds of kB, and fresh allocations of that size
// are page-faulted mappings whose setup serialises the threads in the kernel.
struct ThreadBuffers {
  std::string raw, doc, text;
};
thread_local ThreadBuffers tls;

// ---- libdeflate (when the system has it): whole-buffer gzip inflate, 2-3x zlib's speed ----
// Bound at run time through dlopen so that the library stays optional; PFE_NO_LIBDEFLATE=1
// keeps zlib (A/B runs and tests).  Any result other than success falls back to the zlib
// path, so malformed files fail exactly as before.
struct Deflate {
  using alloc_t = void* (*)();
  using free_t = void (*)(void*);
  using gz_t = int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);
  alloc_t alloc = nullptr;
  free_t release = nullptr;
  gz_t gzip_ex = nullptr;
  Deflate() {
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = (alloc_t)dlsym(h, "libdeflate_alloc_decompressor");
    release = (free_t)dlsym(h, "libdeflate_free_decompressor");
    gzip_ex = (gz_t)dlsym(h, "libdeflate_gzip_decompress_ex");
    if (!alloc || !release || !gzip_ex) alloc = nullptr;
  }
};
const Deflate& deflate_lib() {
  static const Deflate d;
  return d;
}
struct ThreadDecompressor {
  void* d = nullptr;
  ~ThreadDecompressor() {
    if (d) deflate_lib().release(d);
  }
};
thread_local ThreadDecompressor tls_dec;

// all gzip members of raw into out[0, used); false: let zlib decide
bool inflate_libdeflate(const std::string& raw, std::string& out, size_t& used) {
  const Deflate& L = deflate_lib();
  if (!L.alloc) return false;
  const char* e = std::getenv("PFE_NO_LIBDEFLATE");
  if (e && e[0] == '1') return false;
  if (!tls_dec.d) tls_dec.d = L.alloc();
  if (!tls_dec.d) return false;
  size_t pos = 0;
  used = 0;
  for (;;) {
    size_t in_used = 0, out_used = 0;
    int rc;
    for (;;) {
      if (out.size() - used < raw.size() * 4 + (1 << 16))
        out.resize(std::max(out.size() * 2, used + raw.size() * 4 + (1 << 16)));
      rc = L.gzip_ex(tls_dec.d, raw.data() + pos, raw.size() - pos, &out[used], out.size() - used,
                     &in_used, &out_used);
      if (rc != 3) break;  // LIBDEFLATE_INSUFFICIENT_SPACE: a larger buffer, the member again
      out.resize(out.size() * 2);
    }
    if (rc != 0) return false;
    pos += in_used;
    used += out_used;
    // another gzip member may follow; trailing zero padding is tolerated like Python's
    size_t k = pos;
    while (k < raw.size() && raw[k] == 0) ++k;
    if (k == raw.size()) return true;
  }
}

bool read_all(const char* path, bool gz, std::string& out, int& err) {
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    err = PFE_IO_ERR_OPEN;
    return false;
  }
  std::string& raw = tls.raw;
  raw.clear();
  {
    char buf[1 << 16];
    size_t r;
    while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) raw.append(buf, r);
    const bool bad = std::ferror(f);
    std::fclose(f);
    if (bad) {
      err = PFE_IO_ERR_OPEN;
      return false;
    }
  }
  if (!gz) {
    out.assign(raw);
    return true;
  }
  // gzip (possibly several members, as Python's gzip module accepts)
  if (raw.size() < 2 || (uint8_t)raw[0] != 0x1f || (uint8_t)raw[1] != 0x8b) {
    err = PFE_IO_ERR_GZIP;
    return false;
  }
  {
    size_t used = 0;
    if (inflate_libdeflate(raw, out, used)) {
      out.resize(used);
      return true;
    }
  }
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, 15 + 32) != Z_OK) {
    err = PFE_IO_ERR_GZIP;
    return false;
  }
  zs.next_in = (Bytef*)raw.data();
  zs.avail_in = (uInt)raw.size();
  // inflate straight into the (reused) output buffer
  size_t used = 0;
  if (out.size() < raw.size() * 4) out.resize(raw.size() * 4);
  for (;;) {
    if (out.size() - used < (1 << 16)) out.resize(out.size() * 2);
    zs.next_out = (Bytef*)&out[used];
    zs.avail_out = (uInt)std::min<size_t>(out.size() - used, 1u << 30);
    const size_t before = zs.avail_out;
    const int rc = inflate(&zs, Z_NO_FLUSH);
    used += before - zs.avail_out;
    if (rc == Z_STREAM_END) {
      if (zs.avail_in == 0) break;
      // another gzip member follows; trailing zero padding is tolerated like Python's
      size_t k = 0;
      while (k < zs.avail_in && zs.next_in[k] == 0) ++k;
      if (k == zs.avail_in) break;
      if (inflateReset(&zs) != Z_OK) {
        inflateEnd(&zs);
        err = PFE_IO_ERR_GZIP;
        return false;
      }
      continue;
    }
    if (rc != Z_OK && !(rc == Z_BUF_ERROR && zs.avail_out == 0)) {
      inflateEnd(&zs);
      err = PFE_IO_ERR_GZIP;
      return false;
    }
  }
  inflateEnd(&zs);
  out.resize(used);
  return true;
}

size_t find_str(const std::string& d, size_t from, const char* s) {
  const size_t p = d.find(s, from);
  return p == std::string::npos ? d.size() : p;
}

bool is_name_char(char c) {
  return !(c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '/' || c == '>');
}

// one forward scan collecting the target leaf elements in document order
void scan(const std::string& d, std::vector<Elem> (&occ)[NTAGS]) {
  const size_t n = d.size();
  size_t i = 0;
  while (i < n) {
    const size_t lt = d.find('<', i);
    if (lt == std::string::npos) break;
    i = lt;
    if (d.compare(i, 4, "<!--") == 0) {
      i = find_str(d, i + 4, "-->") + 3;
      continue;
    }
    if (d.compare(i, 9, "<![CDATA[") == 0) {
      i = find_str(d, i + 9, "]]>") + 3;
      continue;
    }
    if (d.compare(i, 2, "<?") == 0) {
      i = find_str(d, i + 2, "?>") + 2;
      continue;
    }
    if (d.compare(i, 2, "<!") == 0 || d.compare(i, 2, "</") == 0) {
      i = find_str(d, i + 2, ">") + 1;
      continue;
    }
    // start tag
    size_t ne = i + 1;
    while (ne < n && is_name_char(d[ne])) ++ne;
    // end of the tag, honouring quoted attribute values
    size_t gt = ne;
    char q = 0;
    while (gt < n) {
      const char c = d[gt];
      if (q) {
        if (c == q) q = 0;
      } else if (c == '"' || c == '\'') {
        q = c;
      } else if (c == '>') {
        break;
      }
      ++gt;
    }
    if (gt >= n) break;
    const bool self_close = gt > ne && d[gt - 1] == '/';
    int tag = -1;
    const size_t nl = ne - (i + 1);
    for (int t = 0; t < NTAGS; ++t)
      if (std::strlen(kTagNames[t]) == nl && d.compare(i + 1, nl, kTagNames[t]) == 0) tag = t;
    if (tag >= 0) {
      Elem e;
      e.ab = ne;
      e.ae = self_close ? gt - 1 : gt;
      if (!self_close) {
        const size_t tb = gt + 1;
        size_t te = d.find('<', tb);
        if (te == std::string::npos) te = n;
        e.tb = tb;
        e.te = te;
        e.has_text = te > tb;
        // the text must end at this element's own end tag
        const std::string close = std::string("</") + kTagNames[tag];
        if (d.compare(te, close.size(), close) != 0) e.complex = true;
      }
      occ[tag].push_back(e);
    }
    i = gt + 1;
  }
}

// any byte of p[0, n) that element_text must treat specially: non-ASCII, CR or '&' (SSE2)
inline bool has_special(const unsigned char* p, size_t n) {
  const __m128i cr = _mm_set1_epi8('\r'), amp = _mm_set1_epi8('&');
  size_t k = 0;
  int bits = 0;
  for (; k + 16 <= n; k += 16) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + k));
    bits |= _mm_movemask_epi8(_mm_or_si128(v, _mm_or_si128(_mm_cmpeq_epi8(v, cr), _mm_cmpeq_epi8(v, amp))));
  }
  unsigned special = bits != 0;
  for (; k < n; ++k) {
    const unsigned c = p[k];
    special |= (c >= 0x80u) | (c == (unsigned)'\r') | (c == (unsigned)'&');
  }
  return special != 0;
}

// element text as ElementTree delivers it: CRLF / CR -> LF, entities decoded.
// Returns false (fallback) for non-ASCII text or an unknown entity.
bool element_text(const std::string& d, const Elem& e, std::string& out) {
  // fast path: plain ASCII without CR or entities (every PHCX element in practice) is
  // delivered as it stands
  {
    const unsigned char* p = (const unsigned char*)d.data() + e.tb;
    const size_t len = e.te - e.tb;
    if (!has_special(p, len)) {
      out.assign((const char*)p, len);
      return true;
    }
  }
  out.clear();
  out.reserve(e.te - e.tb);
  for (size_t i = e.tb; i < e.te; ++i) {
    const char c = d[i];
    if ((unsigned char)c >= 0x80) return false;
    if (c == '\r') {
      out.push_back('\n');
      if (i + 1 < e.te && d[i + 1] == '\n') ++i;
    } else if (c == '&') {
      const size_t sc = d.find(';', i);
      if (sc == std::string::npos || sc >= e.te) return false;
      const std::string ent = d.substr(i + 1, sc - i - 1);
      long v = -1;
      if (ent == "lt") v = '<';
      else if (ent == "gt") v = '>';
      else if (ent == "amp") v = '&';
      else if (ent == "apos") v = '\'';
      else if (ent == "quot") v = '"';
      else if (ent.size() > 1 && ent[0] == '#') {
        char* endp = nullptr;
        v = (ent[1] == 'x') ? std::strtol(ent.c_str() + 2, &endp, 16) : std::strtol(ent.c_str() + 1, &endp, 10);
        if (!endp || *endp) return false;
      }
      if (v < 1 || v >= 0x80) return false;
      out.push_back((char)v);
      i = sc;
    } else {
      out.push_back(c);
    }
  }
  return true;
}

bool py_space(char c) { return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f); }

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// int(s, 16) for the 1-2 character slices the reference's loops take
bool py_int_hex(const char* s, size_t len, int& v) {
  size_t b = 0, e = len;
  while (b < e && py_space(s[b])) ++b;
  while (e > b && py_space(s[e - 1])) --e;
  if (b == e) return false;
  int sign = 1;
  if (s[b] == '+' || s[b] == '-') {
    sign = s[b] == '-' ? -1 : 1;
    ++b;
  }
  if (b == e) return false;
  int acc = 0;
  for (size_t k = b; k < e; ++k) {
    const int h = hexval(s[k]);
    if (h < 0) return false;
    acc = acc * 16 + h;
  }
  v = sign * acc;
  return true;
}

// hex decode with the reference's loop (PHCXFile.py:144-186, PHCXOperations.py:263-297):
// skip '\n', take text[i:i+2], stop at the first slice int() rejects
struct HexLut {
  int8_t v[256];
  HexLut() {
    for (int c = 0; c < 256; ++c) v[c] = (int8_t)hexval((char)c);
  }
};
const HexLut kHex;

// 16 hex digits at s -> 8 bytes at o (SSE2); false, with nothing written, when any of the
// 16 is not a hex digit ('\n' included): the caller then takes the reference's loop one step
inline bool hex16(const unsigned char* s, uint8_t* o) {
  const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s));
  const __m128i sign = _mm_set1_epi8((char)0x80);
  const __m128i d = _mm_sub_epi8(v, _mm_set1_epi8('0'));                       // '0'..'9'
  const __m128i isd = _mm_cmplt_epi8(_mm_xor_si128(d, sign), _mm_set1_epi8((char)(0x80 + 10)));
  const __m128i l = _mm_sub_epi8(_mm_or_si128(v, _mm_set1_epi8(0x20)), _mm_set1_epi8('a'));
  const __m128i isl = _mm_cmplt_epi8(_mm_xor_si128(l, sign), _mm_set1_epi8((char)(0x80 + 6)));
  if (_mm_movemask_epi8(_mm_or_si128(isd, isl)) != 0xFFFF) return false;
  const __m128i val = _mm_or_si128(_mm_and_si128(isd, d),
                                   _mm_and_si128(isl, _mm_add_epi8(l, _mm_set1_epi8(10))));
  // byte 2k is the high nibble of output k, byte 2k+1 the low one
  const __m128i hi = _mm_slli_epi16(_mm_and_si128(val, _mm_set1_epi16(0x00FF)), 4);
  const __m128i lo = _mm_srli_epi16(val, 8);
  _mm_storel_epi64(reinterpret_cast<__m128i*>(o), _mm_packus_epi16(_mm_or_si128(hi, lo), hi));
  return true;
}

bool hex_decode(const char* t, size_t n, std::vector<uint8_t>& out, int& err) {
  out.resize(n / 2 + 8);
  uint8_t* o = out.data();
  size_t m = 0;
  const unsigned char* s = (const unsigned char*)t;
  size_t i = 0;
  while (i < n) {
    // runs of 16 hex digits: the pairs are consecutive characters, as the loop below takes them
    if (i + 16 <= n && hex16(s + i, o + m)) {
      i += 16;
      m += 8;
      continue;
    }
    if (s[i] == '\n') {
      ++i;
      continue;
    }
    if (i + 1 < n) {
      const int h0 = kHex.v[s[i]], h1 = kHex.v[s[i + 1]];
      if ((h0 | h1) >= 0) {
        o[m++] = (uint8_t)(h0 * 16 + h1);
        i += 2;
        continue;
      }
    }
    int v;
    if (!py_int_hex(t + i, std::min<size_t>(2, n - i), v)) break;
    if (v < 0 || v > 255) {
      err = PFE_IO_ERR_RANGE;
      out.resize(m);
      return false;
    }
    o[m++] = (uint8_t)v;
    i += 2;
  }
  out.resize(m);
  return true;
}

// float(text) for the plain decimal spellings a C library parses identically
bool py_float(const std::string& s, double& v) {
  size_t b = 0, e = s.size();
  while (b < e && py_space(s[b])) ++b;
  while (e > b && py_space(s[e - 1])) --e;
  if (b == e) return false;
  for (size_t k = b; k < e; ++k) {
    const char c = s[k];
    if (!((c >= '0' && c <= '9') || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-'))
      return false;  // inf / nan / underscores: leave to the host's Python parser
  }
  const std::string t = s.substr(b, e - b);
  char* endp = nullptr;
  errno = 0;
  v = std::strtod(t.c_str(), &endp);
  return endp && *endp == 0;
}

bool py_int_attr(const std::string& s, int& v) {
  size_t b = 0, e = s.size();
  while (b < e && py_space(s[b])) ++b;
  while (e > b && py_space(s[e - 1])) --e;
  if (b == e || e - b > 9) return false;
  int acc = 0;
  for (size_t k = b; k < e; ++k) {
    if (s[k] < '0' || s[k] > '9') return false;
    acc = acc * 10 + (s[k] - '0');
  }
  v = acc;
  return true;
}

bool get_attr(const std::string& d, const Elem& e, const char* name, std::string& val) {
  const std::string a = d.substr(e.ab, e.ae - e.ab);
  const size_t nl = std::strlen(name);
  size_t p = 0;
  while ((p = a.find(name, p)) != std::string::npos) {
    const bool start_ok = p == 0 || py_space(a[p - 1]);
    size_t k = p + nl;
    while (k < a.size() && py_space(a[k])) ++k;
    if (start_ok && k < a.size() && a[k] == '=') {
      ++k;
      while (k < a.size() && py_space(a[k])) ++k;
      if (k < a.size() && (a[k] == '"' || a[k] == '\'')) {
        const char q = a[k];
        const size_t ve = a.find(q, k + 1);
        if (ve == std::string::npos) return false;
        val = a.substr(k + 1, ve - k - 1);
        return val.find('&') == std::string::npos;
      }
      return false;
    }
    p += nl;
  }
  return false;
}

void parse_file(const char* path, int mode, Parsed& P) {
  pfe_phcx_info& info = P.info;
  const bool superb = mode == 1 || (mode < 0 && std::strstr(path, ".gz") == nullptr);
  info.superb = superb ? 1 : 0;
  const int sec = superb ? 0 : 1;  // PHCXFile.py:103 / SUPERBPHCXFile.py:103
  info.section = sec;
  std::string& doc = tls.doc;
  int err = 0;
  if (!read_all(path, !superb, doc, err)) {
    info.status = err;
    return;
  }
  std::vector<Elem> occ[NTAGS];
  scan(doc, occ);
  auto need = [&](int t, int k) -> const Elem* {
    if ((int)occ[t].size() <= k) return nullptr;
    return &occ[t][k];
  };
  const Elem* eprof = need(T_PROFILE, sec);
  const Elem* eblk0 = need(T_DATABLOCK, 0);
  const Elem* eblk = need(T_DATABLOCK, sec);
  const Elem* esub = need(T_SUBBANDS, sec);
  const Elem* edmi = need(T_DMINDEX, sec);
  const Elem* escal[4] = {need(T_BARY, sec), need(T_SNR, sec), need(T_DM, sec), need(T_WIDTH, sec)};
  if (!eprof || !eblk0 || !eblk || !esub || !edmi || !escal[0] || !escal[1] || !escal[2] ||
      !escal[3]) {
    info.status = PFE_IO_ERR_XML;
    return;
  }
  const Elem* all[] = {eprof, eblk0, eblk, esub, edmi, escal[0], escal[1], escal[2], escal[3]};
  for (const Elem* e : all)
    if (e->complex) {
      info.status = PFE_IO_ERR_XML;
      return;
    }
  std::string& text = tls.text;
  auto decode = [&](const Elem* e, std::vector<uint8_t>& out) -> bool {
    if (!e->has_text) {  // hex decode of None -> empty (the host parser's convention)
      out.clear();
      return true;
    }
    // plain ASCII without CR or entities (every PHCX element in practice) is decoded where it
    // lies in the document; anything else through element_text first
    const unsigned char* tp = (const unsigned char*)doc.data() + e->tb;
    const size_t tl = e->te - e->tb;
    const char* hp = (const char*)tp;
    size_t hl = tl;
    if (has_special(tp, tl)) {
      if (!element_text(doc, *e, text)) {
        info.status = PFE_IO_ERR_VALUE;
        return false;
      }
      hp = text.data();
      hl = text.size();
    }
    int derr = 0;
    if (!hex_decode(hp, hl, out, derr)) {
      info.status = derr;
      return false;
    }
    return true;
  };
  if (!decode(eprof, P.profile) || !decode(eblk0, P.lyon_dm) || !decode(eblk, P.fit) ||
      !decode(esub, P.sub))
    return;
  // SubBands nBins / nSub and the reshape
  std::string av;
  int nbins = 0, nsub = 0;
  if (!get_attr(doc, *esub, "nBins", av) || !py_int_attr(av, nbins) ||
      !get_attr(doc, *esub, "nSub", av) || !py_int_attr(av, nsub)) {
    info.status = PFE_IO_ERR_VALUE;
    return;
  }
  if ((int64_t)nbins * nsub != (int64_t)P.sub.size()) {
    info.status = PFE_IO_ERR_SHAPE;
    return;
  }
  // DmIndex: tokens terminated by '\n'; dm_start = token[1], dm_end = the last (:172-183)
  double dm_start = 0, dm_end = 0;
  {
    if (!edmi->has_text || !element_text(doc, *edmi, text)) {
      info.status = PFE_IO_ERR_VALUE;
      return;
    }
    std::vector<std::pair<size_t, size_t>> toks;
    size_t b = 0;
    for (size_t k = 0; k < text.size(); ++k)
      if (text[k] == '\n') {
        toks.emplace_back(b, k);
        b = k + 1;
      }
    if (toks.size() < 2 ||
        !py_float(text.substr(toks[1].first, toks[1].second - toks[1].first), dm_start) ||
        !py_float(text.substr(toks.back().first, toks.back().second - toks.back().first), dm_end)) {
      info.status = PFE_IO_ERR_VALUE;
      return;
    }
  }
  double sv[4];
  for (int k = 0; k < 4; ++k) {
    if (!escal[k]->has_text || !element_text(doc, *escal[k], text) || !py_float(text, sv[k])) {
      info.status = PFE_IO_ERR_VALUE;
      return;
    }
  }
  // reduced DM curve: max of the first 127 values of each full 128-chunk (:237-259)
  const int64_t nfull = (int64_t)P.fit.size() / 128;
  P.dmc.resize((size_t)nfull);
  for (int64_t k = 0; k < nfull; ++k) {
    const uint8_t* c = P.fit.data() + k * 128;
    uint8_t mx = 0;  // max(chunk[:127]) of bytes (a plain loop the compiler vectorises)
    for (int b = 0; b < 127; ++b) mx = c[b] > mx ? c[b] : mx;
    P.dmc[(size_t)k] = (double)mx;
  }
  info.lp = (int32_t)P.profile.size();
  info.nsub = nsub;
  info.lsb = nbins;
  info.ndm = (int32_t)nfull;
  info.ld = (int64_t)P.lyon_dm.size();
  info.lfit = (int64_t)P.fit.size();
  info.scal[0] = sv[0] * 1000;  // BaryPeriod * 1000 (PHCXOperations.py:107)
  info.scal[1] = sv[1];
  info.scal[2] = sv[2];
  info.scal[3] = sv[3];
  info.scal[4] = dm_start;
  info.scal[5] = dm_end;
  info.scal[6] = (double)P.fit.size();
  info.scal[7] = 0.0;
  info.status = PFE_IO_OK;
}

template <class F>
void parallel_for(int64_t n, int nthreads, F&& fn) {
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  nthreads = (int)std::min<int64_t>(nthreads, std::max<int64_t>(1, n));
  std::atomic<int64_t> next{0};
  auto work = [&] {
    for (int64_t i; (i = next.fetch_add(1)) < n;) fn(i);
  };
  if (nthreads == 1) {
    work();
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nthreads);
  for (int t = 0; t < nthreads; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
}

// ---- score text (pfe_format_rows) ----
// str.replace(pat, "0"): left to right, non-overlapping, as Python does.
void replace_with_zero(const std::string& in, const char* pat, std::string& out) {
  out.clear();
  size_t i = 0;
  while (i < in.size()) {
    if (i + 3 <= in.size() && in[i] == pat[0] && in[i + 1] == pat[1] && in[i + 2] == pat[2]) {
      out += '0';
      i += 3;
    } else {
      out += in[i++];
    }
  }
}

void append_clean_name(std::string& s, const char* p, size_t n) {
  thread_local std::string a, b;
  a.assign(p, n);
  replace_with_zero(a, "nan", b);
  replace_with_zero(b, "inf", a);
  s += a;
}

// Python 2.7 str(float) ('%.12g' + ".0" for integral text), then the writers' nan/inf -> 0.
void append_py2_value(std::string& s, double x) {
  if (std::isnan(x)) {
    s += '0';
    return;
  }
  if (std::isinf(x)) {
    s += x > 0 ? "0" : "-0";
    return;
  }
  // std::to_chars(general, 12) is specified as printf's %.12g in the C locale, and is ~4x
  // faster than snprintf (the text of 22 scores per line is the largest host cost of a
  // streamed run after parsing)
  char tmp[40];
  const int k = (int)(std::to_chars(tmp, tmp + sizeof tmp, x, std::chars_format::general, 12).ptr - tmp);
  s.append(tmp, (size_t)k);
  if (!std::memchr(tmp, '.', (size_t)k) && !std::memchr(tmp, 'e', (size_t)k)) s += ".0";
}

}  // namespace

struct pfe_phcx_batch {
  std::vector<Parsed> files;
};

extern "C" {

int pfe_phcx_parse(const char* const* paths, int64_t n, int32_t mode, int32_t nthreads,
                   pfe_phcx_batch** out) {
  if (!out || n < 0 || (n > 0 && !paths) || mode < -1 || mode > 1) return PFE_EINVAL;
  *out = nullptr;
  for (int64_t i = 0; i < n; ++i)
    if (!paths[i]) return PFE_EINVAL;
  auto* b = new (std::nothrow) pfe_phcx_batch;
  if (!b) return PFE_EINVAL;
  b->files.resize((size_t)n);
  parallel_for(n, nthreads, [&](int64_t i) { parse_file(paths[i], mode, b->files[(size_t)i]); });
  *out = b;
  return PFE_OK;
}

int64_t pfe_phcx_count(const pfe_phcx_batch* b) { return b ? (int64_t)b->files.size() : 0; }

int pfe_phcx_info_get(const pfe_phcx_batch* b, int64_t i, pfe_phcx_info* info) {
  if (!b || !info || i < 0 || i >= (int64_t)b->files.size()) return PFE_EINVAL;
  *info = b->files[(size_t)i].info;
  return PFE_OK;
}

int pfe_phcx_fetch(const pfe_phcx_batch* b, int64_t i, int32_t field, void* dst,
                   int64_t capacity) {
  if (!b || !dst || i < 0 || i >= (int64_t)b->files.size()) return PFE_EINVAL;
  const Parsed& P = b->files[(size_t)i];
  if (P.info.status != PFE_IO_OK) return PFE_EINVAL;
  const void* src = nullptr;
  size_t cnt = 0, esz = 1;
  switch (field) {
    case PFE_PHCX_PROFILE: src = P.profile.data(); cnt = P.profile.size(); break;
    case PFE_PHCX_LYON_DM: src = P.lyon_dm.data(); cnt = P.lyon_dm.size(); break;
    case PFE_PHCX_SUBBANDS: src = P.sub.data(); cnt = P.sub.size(); break;
    case PFE_PHCX_DM_CURVE: src = P.dmc.data(); cnt = P.dmc.size(); esz = sizeof(double); break;
    case PFE_PHCX_FIT_BLOCK: src = P.fit.data(); cnt = P.fit.size(); break;
    default: return PFE_EINVAL;
  }
  if ((int64_t)cnt > capacity) return PFE_EINVAL;
  if (cnt) std::memcpy(dst, src, cnt * esz);
  return PFE_OK;
}

int pfe_phcx_pack(const pfe_phcx_batch* b, const int64_t* rows, int64_t nrows, int32_t nthreads,
                  uint8_t* prof, int64_t prof_stride, uint8_t* lyon_dm, int64_t dm_stride,
                  uint8_t* sub, int64_t sub_stride, double* dmcurve, int64_t dmc_stride,
                  double* scal) {
  if (!b || nrows < 0 || (nrows > 0 && !rows)) return PFE_EINVAL;
  for (int64_t r = 0; r < nrows; ++r) {
    const int64_t i = rows[r];
    if (i < 0 || i >= (int64_t)b->files.size()) return PFE_EINVAL;
    const Parsed& P = b->files[(size_t)i];
    if (P.info.status != PFE_IO_OK) return PFE_EINVAL;
    if ((prof && (int64_t)P.profile.size() > prof_stride) ||
        (lyon_dm && (int64_t)P.lyon_dm.size() > dm_stride) ||
        (sub && (int64_t)P.sub.size() > sub_stride) ||
        (dmcurve && (int64_t)P.dmc.size() > dmc_stride))
      return PFE_EINVAL;
  }
  parallel_for(nrows, nthreads, [&](int64_t r) {
    const Parsed& P = b->files[(size_t)rows[r]];
    if (prof && !P.profile.empty()) std::memcpy(prof + r * prof_stride, P.profile.data(), P.profile.size());
    if (lyon_dm && !P.lyon_dm.empty())
      std::memcpy(lyon_dm + r * dm_stride, P.lyon_dm.data(), P.lyon_dm.size());
    if (sub && !P.sub.empty()) std::memcpy(sub + r * sub_stride, P.sub.data(), P.sub.size());
    if (dmcurve && !P.dmc.empty())
      std::memcpy(dmcurve + r * dmc_stride, P.dmc.data(), P.dmc.size() * sizeof(double));
    if (scal) std::memcpy(scal + r * 8, P.info.scal, 8 * sizeof(double));
  });
  return PFE_OK;
}

void pfe_phcx_free(pfe_phcx_batch* b) { delete b; }

int pfe_phcx_info_all(const pfe_phcx_batch* b, pfe_phcx_info* out, int64_t capacity) {
  if (!b || capacity < (int64_t)b->files.size() || (!out && !b->files.empty())) return PFE_EINVAL;
  for (size_t i = 0; i < b->files.size(); ++i) out[i] = b->files[i].info;
  return PFE_OK;
}

int pfe_format_rows(const char* name_blob, const int64_t* name_off, const double* vals,
                    int64_t n, int32_t width, int64_t stride, int32_t style,
                    const uint8_t* skip, int32_t nthreads, char* buf, int64_t cap,
                    int64_t* len) {
  if (n < 0 || width < 0 || style < 0 || style > 2 || !len || (n > 0 && (!vals || !buf)) ||
      (style != 2 && n > 0 && (!name_blob || !name_off)) || stride < width)
    return PFE_EINVAL;
  *len = 0;
  if (n == 0) return PFE_OK;
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  const int64_t nt = std::min<int64_t>(nthreads, std::max<int64_t>(1, n / 256));
  std::vector<std::string> part((size_t)nt);
  auto work = [&](int64_t t) {
    const int64_t r0 = n * t / nt, r1 = n * (t + 1) / nt;
    std::string& s = part[(size_t)t];
    s.reserve((size_t)(r1 - r0) * (size_t)(24 * width + 80));
    for (int64_t r = r0; r < r1; ++r) {
      if (skip && skip[r]) continue;
      if (style == 0) {
        append_clean_name(s, name_blob + name_off[r], (size_t)(name_off[r + 1] - name_off[r]));
        s += ',';
      }
      const double* v = vals + r * stride;
      for (int32_t k = 0; k < width; ++k) {
        if (k) s += ',';
        append_py2_value(s, v[k]);
      }
      if (style == 1) {
        s += ",?%";
        append_clean_name(s, name_blob + name_off[r], (size_t)(name_off[r + 1] - name_off[r]));
      }
      s += '\n';
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    th.reserve((size_t)nt);
    for (int64_t t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& t : th) t.join();
  }
  int64_t total = 0;
  for (const auto& s : part) total += (int64_t)s.size();
  if (total > cap) return PFE_EINVAL;
  char* p = buf;
  for (const auto& s : part) {
    std::memcpy(p, s.data(), s.size());
    p += s.size();
  }
  *len = total;
  return PFE_OK;
}

}  // extern "C"

"""PHCX / SUPERB-PHCX candidate files: host-side parser and synthetic writer.

Parser semantics follow the reference (paths relative to PulsarFeatureExtractor/src/):
  * PHCX (HTRU): gzip XML, scored section 1, 128-bin profile    PHCXFile.py:80,103
  * SUPERB PHCX: plain XML, scored section 0, 64-bin profile    SUPERBPHCXFile.py:80,103
  * Profile hex decode (02X; skip '\\n' only; stop at the first pair int() rejects)
                                                               PHCXFile.py:144-186
  * DataBlock / SubBands hex decode (same rule)                 PHCXOperations.py:263-297,353-383
  * Lyon DM array = decoded DataBlock of XML section 0           PHCXOperations.py:528-539
  * Reduced DM curve: max of the first 127 of each 128 values   PHCXOperations.py:237-259
  * DmIndex: text split on '\\n'; dm_start = token[1], dm_end = last newline-terminated
    token                                                       PHCXOperations.py:172-183
  * Scalars Snr / Dm / BaryPeriod*1000 / Width of the scored section   PHCXOperations.py:107-110

The parser uses xml.etree (C accelerated) instead of minidom; ``getElementsByTagName(t)[i]``
is ``list(root.iter(t))[i]`` and ``childNodes[0].data`` is ``element.text`` for these leaf
elements.
"""
from __future__ import annotations

import gzip
import re
import xml.etree.ElementTree as ET

import numpy as np

_HEXPAIR_OK = re.compile(r"^[0-9A-Fa-f]*$")


def hex_decode(text: str) -> np.ndarray:
    """Decode 02X text exactly as the reference's per-character loops do.

    Fast path: every '\\n'-separated line has an even number of hex digits, so the loop
    simply consumes aligned pairs.  Otherwise fall back to the reference's loop verbatim
    in behaviour (a pair is ``text[i:i+2]`` passed to ``int(.., 16)``, which tolerates
    surrounding whitespace; decoding stops at the first ValueError)."""
    if text is None:
        return np.zeros(0, dtype=np.int64)
    lines = text.split("\n")
    if all(len(s) % 2 == 0 and _HEXPAIR_OK.match(s) for s in lines):
        return np.frombuffer(bytes.fromhex("".join(lines)), dtype=np.uint8).astype(np.int64)
    out = []
    i, n = 0, len(text)
    while i < n:
        if text[i] != "\n":
            try:
                out.append(int(text[i:i + 2], 16))
                i += 2
            except ValueError:
                break
        else:
            i += 1
    return np.asarray(out, dtype=np.int64)


def reduce_dm_curve(block: np.ndarray):
    """PHCXOperations.dm_curve (:237-259): y_k = max(first 127 values of 128-chunk k),
    x_k = 128k - 1 (the chunk's last index minus 128).  A trailing partial chunk is
    dropped."""
    nfull = len(block) // 128
    if nfull == 0:
        return np.zeros(0, dtype=np.float64), np.zeros(0, dtype=np.float64)
    chunks = np.asarray(block[: nfull * 128]).reshape(nfull, 128)
    y = chunks[:, :127].max(axis=1).astype(np.float64)
    x = (np.arange(nfull) * 128 + 127 - 128).astype(np.float64)
    return y, x


def parse_dm_index(text: str):
    """(dm_start, dm_end) from the DmIndex text (PHCXOperations.py:172-182)."""
    toks = []
    tmp = ""
    for ch in text:
        if ch != "\n":
            tmp += ch
        else:
            toks.append(tmp)
            tmp = ""
    return float(toks[1]), float(toks[len(toks) - 1])


class PHCXCandidate:
    """Arrays of one parsed candidate (what the batch packer hands to libpfe)."""

    __slots__ = ("path", "superb", "section", "profile", "lyon_dm", "subbands",
                 "dm_curve", "scal", "period_ms", "snr", "dm", "width")

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)


def _read_xml(path: str, superb: bool):
    if superb:
        with open(path, "rb") as f:
            data = f.read()
    else:
        with gzip.open(path, "rb") as f:
            data = f.read()
    return ET.fromstring(data)


def band_rows(path: str, tag: str, superb: bool | None = None) -> np.ndarray:
    """PHCXOperations.getSubbandData / getSubintData (:434-438, :479-483): the hex block of
    ``getElementsByTagName(tag)[1]`` (always element 1) as an (nSub, nBins) integer array
    (hexToDec :353-383).  IndexError when the file has fewer than two such elements."""
    if superb is None:
        superb = ".gz" not in path
    root = _read_xml(path, superb)
    el = list(root.iter(tag))[1]
    return hex_decode(el.text).reshape(int(el.get("nSub")), int(el.get("nBins")))


def parse(path: str, superb: bool | None = None) -> PHCXCandidate:
    """Parse a PHCX (gzip) or SUPERB PHCX file the way Candidate.py:141-150 dispatches:
    names containing '.gz' are HTRU PHCX (section 1), anything else SUPERB (section 0)."""
    if superb is None:
        superb = ".gz" not in path
    return _from_root(_read_xml(path, superb), 0 if superb else 1, path)


def parse_document(doc, section: int) -> PHCXCandidate:
    """A candidate from the XML the reference's own objects hold: the minidom Document that
    PHCXFile.load keeps in self.rawdata and hands to PHCXOperations (PHCXFile.py:103-104,
    :454-654), or its text / bytes; `section` is the reference's argument (1 HTRU PHCX, 0
    SUPERB), which selects the k-th occurrence of every tag as getElementsByTagName(tag)[k]
    does."""
    if hasattr(doc, "toxml"):
        doc = doc.toxml(encoding="utf-8")
    root = ET.fromstring(doc)
    return _from_root(root, int(section), "")


def _from_root(root, sec: int, path: str) -> PHCXCandidate:
    superb = sec == 0

    def elems(tag):
        return list(root.iter(tag))

    def fval(tag):
        return float(elems(tag)[sec].text)

    profile = hex_decode(elems("Profile")[sec].text)
    blocks = elems("DataBlock")
    lyon_dm = hex_decode(blocks[0].text)  # getDMCurveData always reads section 0 (:538)
    fit_block = hex_decode(blocks[sec].text)
    y, _x = reduce_dm_curve(fit_block)
    sb = elems("SubBands")[sec]
    nbins = int(sb.get("nBins"))
    nsub = int(sb.get("nSub"))
    subbands = hex_decode(sb.text).reshape(nsub, nbins)
    dm_start, dm_end = parse_dm_index(elems("DmIndex")[sec].text)
    period_ms = fval("BaryPeriod") * 1000
    snr, dmv, width = fval("Snr"), fval("Dm"), fval("Width")
    scal = np.array([period_ms, snr, dmv, width, dm_start, dm_end, float(len(fit_block)), 0.0])
    return PHCXCandidate(path=path, superb=superb, section=sec, profile=profile,
                         lyon_dm=lyon_dm, subbands=subbands, dm_curve=y, scal=scal,
                         period_ms=period_ms, snr=snr, dm=dmv, width=width)


def is_valid(path: str, superb: bool | None = None) -> bool:
    """PHCXFile.isValid (PHCXFile.py:190-287) / SUPERBPHCXFile.isValid (SUPERBPHCXFile.py:
    190-): the reference's well-formedness test of a candidate file, run only in debug (-v)
    mode (PHCXFile.load :108-118).  False: the three block tags do not occur exactly twice,
    the section-1 profile text is <= 100 characters or the sub-band / DataBlock texts
    <= 1000, SubBands[1] is not nBins = 128 (64 for SUPERB) x nSub = 16, or the DmIndex[1]
    text is <= 100 characters.  The NaN test (:250) compares floats with the string "nan"
    and never fails, but its float() of Width / Snr / Dm / BaryPeriod[1] can raise, and so
    can a missing element: those exceptions propagate as in the reference."""
    if superb is None:
        superb = ".gz" not in path
    root = _read_xml(path, superb)

    def elems(tag):
        return list(root.iter(tag))

    def text(el):  # minidom childNodes[0].data: IndexError for an empty element
        if el.text is None:
            raise IndexError("list index out of range")
        return el.text

    prof, sub, blk = elems("Profile"), elems("SubBands"), elems("DataBlock")
    if not (len(prof) == len(sub) == len(blk) == 2):
        return False
    sub_fft, blk_fft = text(sub[0]), text(blk[0])  # noqa: F841 (read as the reference does)
    prof_opt, sub_opt, blk_opt = text(prof[1]), text(sub[1]), text(blk[1])
    if not (len(prof_opt) > 100 and len(sub_opt) > 1000 and len(sub_fft) > 1000 and
            len(blk_opt) > 1000):
        return False
    nbins, nsub = int(sub[1].get("nBins")), int(sub[1].get("nSub"))
    ndmi = len(text(elems("DmIndex")[1]))
    if not (nbins == (64 if superb else 128) and nsub == 16 and ndmi > 100):
        return False
    for tag in ("Width", "Snr", "Dm", "BaryPeriod"):
        float(text(elems(tag)[1]))
    return True


# ---------------------------------------------------------------------------------------
# synthetic writer (fixtures, tests, CLI demos)
# ---------------------------------------------------------------------------------------
def _hex_lines(values, per_line: int = 32) -> str:
    s = "".join("%02X" % int(v) for v in values)
    step = 2 * per_line
    return "\n" + "\n".join(s[i:i + step] for i in range(0, len(s), step)) + "\n"


def make_datablock(curve: np.ndarray, rng: np.random.Generator) -> np.ndarray:
    """A DataBlock whose reduced DM curve (max of the first 127 of each 128) is `curve`:
    chunk k holds values <= curve[k] with curve[k] at a random position among the first
    127, and a random (possibly larger) value in the dropped 128th slot."""
    nd = len(curve)
    blk = np.empty((nd, 128), dtype=np.int64)
    for k, v in enumerate(curve.astype(np.int64)):
        blk[k, :] = rng.integers(0, v + 1, size=128)
        blk[k, rng.integers(0, 127)] = v
        blk[k, 127] = rng.integers(0, 256)
    return blk.reshape(-1)


def write(path: str, *, profile, subbands, datablocks, dm_start, dm_end, n_dm_index,
          period_s, snr, dm, width, superb: bool = False, subints=None):
    """Write a synthetic candidate with two <Section>s.

    Both sections carry the same profile, sub-bands, DmIndex and best values (and, when
    ``subints`` (nsubint x nbins) is given, the same <SubIntegrations> block);
    ``datablocks = (block0, block1)`` are the two sections' DataBlocks.  The Lyon DM array
    is always block0 (PHCXOperations.py:538); the DM-curve fit reads the scored section's
    block (1 for PHCX, 0 for SUPERB).  Returns the scored section index."""
    sec = 0 if superb else 1
    prof = np.asarray(profile)
    sbs = np.asarray(subbands)
    nsub, nb = sbs.shape
    dm_idx = np.linspace(dm_start, dm_end, n_dm_index)
    dmtext = "\n" + "\n".join(repr(float(v)) for v in dm_idx) + "\n"
    parts = ["<?xml version='1.0'?>\n<phcf>\n"]
    for s_ in range(2):
        blk = datablocks[s_]
        parts.append(f"<Section name='{'FFT' if s_ == 0 else 'FFT-pdmpd'}'>\n")
        parts.append(f"<BestValues>\n<BaryPeriod>{period_s!r}</BaryPeriod>\n<Dm>{dm!r}</Dm>\n"
                     f"<Snr>{snr!r}</Snr>\n<Width>{width!r}</Width>\n</BestValues>\n")
        parts.append(f"<SubBands nBins='{nb}' nSub='{nsub}' format='02X'>"
                     f"{_hex_lines(sbs.reshape(-1))}</SubBands>\n")
        if subints is not None:
            si = np.asarray(subints)
            parts.append(f"<SubIntegrations nBins='{si.shape[1]}' nSub='{si.shape[0]}' "
                         f"format='02X'>{_hex_lines(si.reshape(-1))}</SubIntegrations>\n")
        parts.append(f"<Profile nBins='{len(prof)}' format='02X'>{_hex_lines(prof)}</Profile>\n")
        parts.append(f"<DmCurve><DmIndex>{dmtext}</DmIndex></DmCurve>\n")
        parts.append(f"<DataBlock format='02X'>{_hex_lines(blk)}</DataBlock>\n")
        parts.append("</Section>\n")
    parts.append("</phcf>\n")
    data = "".join(parts).encode()
    if superb:
        with open(path, "wb") as f:
            f.write(data)
    else:
        with gzip.open(path, "wb") as f:
            f.write(data)
    return sec

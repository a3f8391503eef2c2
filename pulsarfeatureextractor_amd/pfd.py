"""PRESTO .pfd candidate files: host-side reader and synthetic writer.

Reader semantics follow PFDFile.load (PulsarFeatureExtractor/src/PFDFile.py:96-252):
  * byte order: little-endian unless one of the first five int32 exceeds 100000 in
    magnitude, then big-endian (:113-118)
  * header ints, four length-prefixed strings, an optional 16+16-byte RA/Dec block (present
    when the next 16 bytes are all in '0123456789:.-\\0', :126-141), doubles/floats of the
    fold, dms / periods / pdots, profs[npart][nsub][proflen] and foldstats[npart][nsub][7]
  * derived quantities: binspersec = fold_p1 * proflen, chanpersub = numchan // nsub (Py2
    integer '/'), subfreqs, avgprof = (profs / proflen).sum(), varprof = sum of the
    prof_var foldstats (:219-252, calc_varprof :314-327)
A truncated profs/foldstats block leaves zeros, as the reference's per-row try/except does.
"""
from __future__ import annotations

import struct

import numpy as np

_POSN_CHARS = set(b"0123456789:.-\0")


class PFDData:
    """Header fields and arrays of one .pfd file (the attributes PFDFile.load sets)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def read(path: str) -> PFDData:
    with open(path, "rb") as f:
        data = f.read()
    pos = 0

    def take(n):
        nonlocal pos
        if pos + n > len(data):
            raise struct.error("unpack requires a buffer of %d bytes" % n)
        b = data[pos:pos + n]
        pos += n
        return b

    head = take(20)
    sw = "<"
    if np.abs(np.asarray(struct.unpack("<5i", head), dtype=np.float64)).max() > 100000:
        sw = ">"
    numdms, numperiods, numpdots, nsub, npart = struct.unpack(sw + "5i", head)
    proflen, numchan, pstep, pdstep, dmstep, ndmfact, npfact = struct.unpack(sw + "7i", take(28))
    strs = []
    for _ in range(4):
        (ln,) = struct.unpack(sw + "i", take(4))
        strs.append(take(ln))
    test = take(16)
    if all(c in _POSN_CHARS for c in test):
        rastr = test[: test.find(b"\0")]
        test2 = take(16)
        decstr = test2[: test2.find(b"\0")]
        dt, start_t = struct.unpack(sw + "dd", take(16))
    else:
        rastr = decstr = b"Unknown"
        dt, start_t = struct.unpack(sw + "dd", test)
    end_t, tepoch, bepoch, avgvoverc, lofreq, chan_wid, bestdm = struct.unpack(sw + "7d", take(56))
    vals = {}
    for name in ("topo", "bary", "fold"):
        pw, _tmp = struct.unpack(sw + "2f", take(8))
        p1, p2, p3 = struct.unpack(sw + "3d", take(24))
        vals[name] = (pw, p1, p2, p3)
    orb = struct.unpack(sw + "7d", take(56))
    dms = np.asarray(struct.unpack(sw + "%dd" % numdms, take(8 * numdms)))
    periods = np.asarray(struct.unpack(sw + "%dd" % numperiods, take(8 * numperiods)))
    pdots = np.asarray(struct.unpack(sw + "%dd" % numpdots, take(8 * numpdots)))
    dt_ = np.dtype(np.float64).newbyteorder(sw)
    profs = np.zeros((npart, nsub, proflen), dtype=np.float64)
    nprof = npart * nsub * proflen
    avail = max(0, min(nprof, (len(data) - pos) // 8))
    if sw == "<":
        # row by row: a row that cannot be read completely stays zero (:170-176)
        rows = avail // proflen if proflen else 0
        flat = np.frombuffer(data, dtype=dt_, count=rows * proflen, offset=pos)
        profs.reshape(-1, proflen)[:rows] = flat.reshape(rows, proflen)
        pos += rows * proflen * 8
        if rows < npart * nsub:
            pos = len(data)
    else:
        if avail < nprof:
            raise struct.error("unpack requires a buffer of %d bytes" % (8 * nprof))
        profs[:] = np.frombuffer(data, dtype=dt_, count=nprof, offset=pos).reshape(profs.shape)
        pos += nprof * 8
    stats = np.zeros((npart, nsub, 7), dtype=np.float64)
    for ii in range(npart):
        for jj in range(nsub):
            if pos + 56 <= len(data):
                stats[ii, jj] = np.frombuffer(data, dtype=dt_, count=7, offset=pos)
                pos += 56
    binspersec = vals["fold"][1] * proflen
    chanpersub = numchan // nsub
    subdeltafreq = chan_wid * chanpersub
    losubfreq = lofreq + subdeltafreq - chan_wid
    subfreqs = np.arange(nsub, dtype="d") * subdeltafreq + losubfreq
    varprof = 0.0
    for part in range(npart):
        for sub in range(nsub):
            varprof += stats[part][sub][5]
    return PFDData(
        swap=sw, numdms=numdms, numperiods=numperiods, numpdots=numpdots, nsub=nsub,
        npart=npart, proflen=proflen, numchan=numchan, filenm=strs[0], candnm=strs[1],
        telescope=strs[2], pgdev=strs[3], rastr=rastr, decstr=decstr, dt=dt, startT=start_t,
        endT=end_t, tepoch=tepoch, bepoch=bepoch, avgvoverc=avgvoverc, lofreq=lofreq,
        chan_wid=chan_wid, bestdm=bestdm, topo_p1=vals["topo"][1], bary_p1=vals["bary"][1],
        fold_p1=vals["fold"][1], orb=orb, dms=dms, periods=periods, pdots=pdots, profs=profs,
        stats=stats, binspersec=binspersec, chanpersub=chanpersub, subdeltafreq=subdeltafreq,
        losubfreq=losubfreq, subfreqs=subfreqs, avgprof=(profs / proflen).sum(),
        varprof=varprof)


def write(path: str, *, profs, stats=None, dms, bestdm, fold_p1, bary_p1=None, lofreq=1200.0,
          chan_wid=1.0, numchan=None, dt=6.4e-5, big_endian=False, with_posn=True,
          periods=None, pdots=None):
    """Synthetic .pfd with the PRESTO layout PFDFile.load reads."""
    profs = np.asarray(profs, dtype=np.float64)
    npart, nsub, proflen = profs.shape
    if numchan is None:
        numchan = nsub * 4
    if stats is None:
        stats = np.zeros((npart, nsub, 7))
        stats[:, :, 0] = 1000.0
        stats[:, :, 5] = profs.var(axis=2) * proflen
    if bary_p1 is None:
        bary_p1 = fold_p1
    dms = np.atleast_1d(np.asarray(dms, dtype=np.float64))
    periods = np.asarray([fold_p1] if periods is None else periods, dtype=np.float64)
    pdots = np.asarray([0.0] if pdots is None else pdots, dtype=np.float64)
    sw = ">" if big_endian else "<"
    out = [struct.pack(sw + "5i", len(dms), len(periods), len(pdots), nsub, npart),
           struct.pack(sw + "7i", proflen, numchan, 1, 1, 1, 1, 1)]
    for s in (b"synthetic.dat", b"PSR_SYN", b"Parkes", b"/null"):
        out.append(struct.pack(sw + "i", len(s)) + s)
    if with_posn:
        out.append(b"12:34:56.7890\0\0\0")
        out.append(b"-12:34:56.789\0\0\0")
    out.append(struct.pack(sw + "dd", dt, 0.0))
    out.append(struct.pack(sw + "7d", 1000.0, 56000.0, 56000.5, 0.0, lofreq, chan_wid, bestdm))
    for p1 in (fold_p1, bary_p1, fold_p1):
        out.append(struct.pack(sw + "2f", 1.0, 0.0) + struct.pack(sw + "3d", p1, 0.0, 0.0))
    out.append(struct.pack(sw + "7d", *([0.0] * 7)))
    out.append(struct.pack(sw + "%dd" % len(dms), *dms))
    out.append(struct.pack(sw + "%dd" % len(periods), *periods))
    out.append(struct.pack(sw + "%dd" % len(pdots), *pdots))
    out.append(profs.astype(np.dtype(np.float64).newbyteorder(sw)).tobytes())
    out.append(np.asarray(stats, dtype=np.float64).astype(np.dtype(np.float64).newbyteorder(sw)).tobytes())
    with open(path, "wb") as f:
        f.write(b"".join(out))


def batch_inputs(datas):
    """Dense pfe_pfd_dmprof inputs for PFDData of one (npart, nsub, proflen) shape."""
    n = len(datas)
    d0 = datas[0]
    profs = np.empty((n, d0.npart, d0.nsub, d0.proflen), dtype=np.float64)
    subfreqs = np.empty((n, d0.nsub), dtype=np.float64)
    scal = np.zeros((n, 8), dtype=np.float64)
    for i, d in enumerate(datas):
        profs[i] = d.profs
        subfreqs[i] = d.subfreqs
        dms = np.atleast_1d(d.dms)
        scal[i] = (d.bestdm, d.binspersec, d.avgprof, d.varprof, dms[0], dms[-1], d.numdms,
                   d.bary_p1)
    return profs, subfreqs, scal

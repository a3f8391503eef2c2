"""Drop-in mirror of the reference's second plug-in class, backed by libpfe's per-group entry
points (include/pfe.h: pfe_sinusoid4, pfe_gauss7, pfe_params4, pfe_dmfit4, pfe_subband3).

Reference classes (PulsarFeatureExtractor/src/) and what replaces them here:
  ProfileOperationsInterface  ProfileOperationsInterface.py:38-130 -> ProfileOperationsInterface
  ProfileOperations           ProfileOperations.py:164-          -> ProfileOperations
                              (getSinusoidFittings :190-376, getGaussianFittings :595-770)
  PHCXOperations              PHCXOperations.py:44-             -> PHCXOperations
                              (getCandidateParameters :81-112, getDMFittings :121-233,
                               getSubbandParameters :305-349)

A reference-side subclass that needs one score group (PHCXFile.py:454, :521, :569, :613,
:654 call one method each) binds the matching C-ABI function.  Every method here scores one
candidate (the reference's granularity); the `*_batch` forms take n candidates at once.
Values are the bits of the same group's columns of pfe_bates22 (same kernels); where the
reference raises inside a method, the method raises ``Exception`` with the text PHCXFile
reports for that group (candidate.GROUP_ERRORS).  Profiles are the PHCX byte profiles
(integers 0-255); the PFD path's float profiles go through pfd.py / pfe_pfd_bates22.
"""
from __future__ import annotations

import numpy as np

from . import phcx as _phcx
from ._native import PFE_NSCAL, Engine
from .candidate import get_engine, status_error


class ProfileOperationsInterface:
    """ProfileOperationsInterface.py:38-130: the methods a profile-scoring plug-in provides."""

    def __init__(self, debugFlag=False):
        self.debug = debugFlag

    def getSinusoidFittings(self, profile):
        raise NotImplementedError("Please Implement this method")

    def fitSineSqr(self, yData, maxima):
        raise NotImplementedError("Please Implement this method")

    def getGaussianFittings(self, profile):
        raise NotImplementedError("Please Implement this method")

    def fitGaussian(self, xData, yData):
        raise NotImplementedError("Please Implement this method")

    def fitGaussianFixedWidthBins(self, xData, yData, bins):
        raise NotImplementedError("Please Implement this method")

    def fitGaussianWithBackground(self, xData, yData):
        raise NotImplementedError("Please Implement this method")

    def fitGaussianT1(self, yData):
        raise NotImplementedError("Please Implement this method")

    def fitDoubleGaussianT2(self, yData):
        raise NotImplementedError("Please Implement this method")

    def fitDoubleGaussian(self, yData):
        raise NotImplementedError("Please Implement this method")

    def fitDoubleGaussianWithBackground(self, yData, p0):
        raise NotImplementedError("Please Implement this method")

    def getCandidateParameters(self, profile):
        raise NotImplementedError("Please Implement this method")

    def getDMFittings(self, data):
        raise NotImplementedError("Please Implement this method")

    def getSubbandParameters(self, data=None, profile=None):
        raise NotImplementedError("Please Implement this method")


def _u8_rows(profile) -> np.ndarray:
    p = np.asarray(profile)
    if p.ndim == 1:
        p = p[None, :]
    if p.size and (p.min() < 0 or p.max() > 255 or not np.array_equal(p, np.round(p))):
        raise TypeError("byte profiles (integers 0-255) expected")
    return p.astype(np.uint8)


def _raise_failed(st) -> None:
    for s in np.atleast_1d(np.asarray(st)):
        msg = status_error(int(s))
        if msg:
            raise Exception(msg)


class ProfileOperations(ProfileOperationsInterface):
    """ProfileOperations.py: the score groups computed from the profile alone."""

    def __init__(self, debugFlag=False, engine: Engine | None = None):
        super().__init__(debugFlag)
        self._engine = engine

    @property
    def engine(self) -> Engine:
        return self._engine or get_engine()

    # ---- batched forms: (n, k) scores and (n,) status bits ------------------------------
    def getSinusoidFittings_batch(self, profiles):
        p = _u8_rows(profiles)
        return self.engine.sinusoid4(p, np.zeros((len(p), PFE_NSCAL)))

    def getGaussianFittings_batch(self, profiles):
        p = _u8_rows(profiles)
        return self.engine.gauss7(p, np.zeros((len(p), PFE_NSCAL)))

    # ---- per candidate (the reference's signatures) --------------------------------------
    def getSinusoidFittings(self, profile):
        """:190-376 -> [chi^2 sine / maxima, chi^2 sine^2 / maxima, len(diff), sum residuals]"""
        out, st = self.getSinusoidFittings_batch(profile)
        _raise_failed(st)
        return [float(v) for v in out[0]]

    def getGaussianFittings(self, profile):
        """:595-770 -> scores 5-11."""
        out, st = self.getGaussianFittings_batch(profile)
        _raise_failed(st)
        return [float(v) for v in out[0]]

    # ---- the per-fit methods ---------------------------------------------------------------
    # The reference calls each of these only from inside its group method (getSinusoidFittings
    # :370-371; getGaussianFittings :640-760; fitDoubleGaussian :1330-1420 calls
    # fitDoubleGaussianWithBackground), and the engine runs each fit only as a stage of its
    # group's pooled kernel chain (csrc/bates_sine_dm_sub.hip k_sineg; csrc/bates_gauss.h
    # k_ghistg / k_gfixg / k_gt1g / k_gdgg / k_gdg8g), whose intermediate parameters, fit
    # arrays and FWHMs never leave the device.  So none is a group of its own: each raises,
    # naming the group method (and its columns) that carries the fit's result.
    def _per_fit(self, name, ref, group, cols):
        raise NotImplementedError(
            f"ProfileOperations.{name} ({ref}) is not a score group of its own: the fit runs "
            f"inside {group} (include/pfe.h), whose result is {cols}; call {group} on the "
            f"profile instead")

    def fitSine(self, yData, maxima):
        """ProfileOperations.py:380-491 (chi^2 of the fixed-amplitude sine fit).  Runs inside
        getSinusoidFittings / pfe_sinusoid4: s1 = fitSine(profile, maxima) / maxima with the
        profile's own maxima (:370)."""
        self._per_fit("fitSine", "ProfileOperations.py:380-491", "getSinusoidFittings",
                      "s1 = fitSine(profile, maxima) / maxima")

    def fitSineSqr(self, yData, maxima):
        """:495-587 (chi^2 of the sine^2 fit, its residual sign kept).  Runs inside
        getSinusoidFittings / pfe_sinusoid4: s2 = fitSineSqr(profile, maxima) / maxima (:371)."""
        self._per_fit("fitSineSqr", "ProfileOperations.py:495-587", "getSinusoidFittings",
                      "s2 = fitSineSqr(profile, maxima) / maxima")

    def fitGaussian(self, xData, yData):
        """:774-983 (Gaussian fit to a Freedman-Diaconis histogram: of the profile's
        derivative and of the profile, :660, :681).  Runs inside getGaussianFittings /
        pfe_gauss7 (k_ghistg): s5-s7 (:720-722)."""
        self._per_fit("fitGaussian", "ProfileOperations.py:774-983", "getGaussianFittings",
                      "s5-s7 (columns 0-2 of pfe_gauss7)")

    def fitGaussianFixedWidthBins(self, xData, yData, bins):
        """:988-1057 (the fixed-centre fit to the profile histogram, :701).  Runs inside
        getGaussianFittings / pfe_gauss7 (k_gfixg): s5, s6."""
        self._per_fit("fitGaussianFixedWidthBins", "ProfileOperations.py:988-1057",
                      "getGaussianFittings", "s5-s6 (columns 0-1 of pfe_gauss7)")

    def fitGaussianWithBackground(self, xData, yData):
        """:1194-1264 (Gaussian plus background).  Runs inside getGaussianFittings /
        pfe_gauss7 (k_gt1g, called by fitGaussianT1 :1123): s8, s9."""
        self._per_fit("fitGaussianWithBackground", "ProfileOperations.py:1194-1264",
                      "getGaussianFittings", "s8-s9 (columns 3-4 of pfe_gauss7)")

    def fitGaussianT1(self, yData):
        """:1061-1132 (the T1 fit).  Runs inside getGaussianFittings / pfe_gauss7 (k_gt1g):
        s8, s9."""
        self._per_fit("fitGaussianT1", "ProfileOperations.py:1061-1132", "getGaussianFittings",
                      "s8-s9 (columns 3-4 of pfe_gauss7)")

    def fitDoubleGaussianT2(self, yData):
        """:1136-1190 (the T2 double-Gaussian test).  Runs inside getGaussianFittings /
        pfe_gauss7 (k_gdgg peel passes + k_gdg8g): s10, s11."""
        self._per_fit("fitDoubleGaussianT2", "ProfileOperations.py:1136-1190",
                      "getGaussianFittings", "s10-s11 (columns 5-6 of pfe_gauss7)")

    def fitDoubleGaussian(self, yData):
        """:1268-1428 (peel passes, then the 8-parameter fit and the combination rule; called
        by fitDoubleGaussianT2 :1183).  Runs inside getGaussianFittings / pfe_gauss7 (k_gdgg +
        k_gdg8g): s10, s11."""
        self._per_fit("fitDoubleGaussian", "ProfileOperations.py:1268-1428",
                      "getGaussianFittings", "s10-s11 (columns 5-6 of pfe_gauss7)")

    def fitDoubleGaussianWithBackground(self, yData, p0):
        """:1432-1483 (the 8-parameter fit from fitDoubleGaussian's start point, :1411).  Runs inside
        getGaussianFittings / pfe_gauss7 (k_gdg8g): s10, s11."""
        self._per_fit("fitDoubleGaussianWithBackground", "ProfileOperations.py:1432-1483",
                      "getGaussianFittings", "s10-s11 (columns 5-6 of pfe_gauss7)")


class PHCXOperations(ProfileOperations):
    """PHCXOperations.py: the groups read from the candidate file itself.  `data` is what the
    reference passes -- its minidom Document (PHCXFile.rawdata) or that XML's text, read at
    `section` -- or a parsed candidate (phcx.parse) or a candidate path, whose `section` is
    checked against the file type (1 PHCX, 0 SUPERB)."""

    @staticmethod
    def _cand(data, section=None):
        if isinstance(data, str):
            c = _phcx.parse(data)
        elif hasattr(data, "toxml") or isinstance(data, (bytes, bytearray)):
            # the reference's own xmldata (minidom Document, PHCXFile.py:103-104) or its text
            c = _phcx.parse_document(data, 1 if section is None else section)
        else:
            c = data
        if section is not None and int(section) != c.section:
            raise ValueError(f"section {section}: this candidate is read from section {c.section}")
        return c

    def getCandidateParameters_batch(self, scal):
        return self.engine.params4(np.asarray(scal, dtype=np.float64))

    def getDMFittings_batch(self, dmcurves, scal):
        return self.engine.dmfit4(np.asarray(dmcurves, dtype=np.float64),
                                  np.asarray(scal, dtype=np.float64))

    def getSubbandParameters_batch(self, profiles, subbands, scal):
        return self.engine.subband3(_u8_rows(profiles), np.asarray(subbands, dtype=np.uint8),
                                    np.asarray(scal, dtype=np.float64))

    def getCandidateParameters(self, data, section=None):
        """:81-112 -> [period (ms), snr, dm, width] as the method returns them (PHCXFile
        applies filterScore(13/14) when it stores s13/s14)."""
        c = self._cand(data, section)
        out, _st = self.getCandidateParameters_batch(c.scal[None, :])
        return [float(v) for v in out[0]]

    def getDMFittings(self, data, section=None):
        """:121-233 -> [peak, |1 - Prop|, Shift, chi_theo] (s18 = filterScore(18, Shift))."""
        c = self._cand(data, section)
        if len(c.dm_curve) < 3:  # leastsq with fewer rows than parameters raises
            raise Exception(status_error(0x004))
        out, st = self.getDMFittings_batch(c.dm_curve[None, :], c.scal[None, :])
        _raise_failed(st)
        return tuple(float(v) for v in out[0])  # the reference returns a tuple (:233)

    def getSubbandParameters(self, section=None, data=None, profile=None):
        """:305-349 -> [RMS of peak positions, mean pair correlation, correlation integral]
        ([0.0, 0.0, 0.0] without data and profile, :331-332)."""
        if data is None and profile is None:
            return [0.0, 0.0, 0.0]
        c = self._cand(data, section)
        prof = c.profile if profile is None else profile
        out, st = self.getSubbandParameters_batch(prof, c.subbands[None], c.scal[None, :])
        _raise_failed(st)
        return [float(v) for v in out[0]]

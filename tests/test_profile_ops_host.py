"""Host side of the ProfileOperationsInterface mirror (pulsarfeatureextractor_amd.profile_ops):
the abstract interface raises like the reference's, byte profiles are validated, and every
per-group entry point is declared and bound (no compute calls without a GPU)."""
import numpy as np
import pytest

from pulsarfeatureextractor_amd import _native, profile_ops


def test_interface_is_abstract_like_the_reference():
    iface = profile_ops.ProfileOperationsInterface(False)
    for name, args in (("getSinusoidFittings", ([1, 2],)), ("getGaussianFittings", ([1],)),
                       ("getCandidateParameters", ([1],)), ("getDMFittings", (None,)),
                       ("getSubbandParameters", ()), ("fitSineSqr", ([1], 1)),
                       ("fitDoubleGaussianWithBackground", ([1], None))):
        with pytest.raises(NotImplementedError, match="Please Implement this method"):
            getattr(iface, name)(*args)


def test_byte_profiles_only():
    assert profile_ops._u8_rows([0, 255, 7]).dtype == np.uint8
    assert profile_ops._u8_rows(np.arange(6).reshape(2, 3)).shape == (2, 3)
    for bad in ([0.5, 1], [-1, 3], [256, 0]):
        with pytest.raises(TypeError):
            profile_ops._u8_rows(bad)


def test_group_entry_points_bound():
    lib = _native.load_library()
    for s in ("pfe_sinusoid4", "pfe_gauss7", "pfe_params4", "pfe_dmfit4", "pfe_subband3"):
        assert s in _native.EXPORTED_SYMBOLS and hasattr(lib, s)
    for m in ("sinusoid4", "gauss7", "params4", "dmfit4", "subband3"):
        assert callable(getattr(_native.Engine, m))


def test_per_fit_methods_point_at_their_group():
    """The reference's per-fit methods (ProfileOperations.py:380-1483) run only inside a group
    here: each raises with the group method that carries its result, not the interface stub."""
    ops = profile_ops.ProfileOperations(False)
    for name, args, group in (("fitSine", ([1, 2], 1), "getSinusoidFittings"),
                              ("fitSineSqr", ([1, 2], 1), "getSinusoidFittings"),
                              ("fitGaussian", ([0], [1]), "getGaussianFittings"),
                              ("fitGaussianFixedWidthBins", ([0], [1], 4), "getGaussianFittings"),
                              ("fitGaussianWithBackground", ([0], [1]), "getGaussianFittings"),
                              ("fitGaussianT1", ([1],), "getGaussianFittings"),
                              ("fitDoubleGaussianT2", ([1],), "getGaussianFittings"),
                              ("fitDoubleGaussian", ([1],), "getGaussianFittings"),
                              ("fitDoubleGaussianWithBackground", ([1], None), "getGaussianFittings")):
        with pytest.raises(NotImplementedError, match=group) as e:
            getattr(ops, name)(*args)
        assert "Please Implement" not in str(e.value) and name in str(e.value)


def test_subband_parameters_without_data():
    """getSubbandParameters(section) with neither data nor profile is [0.0, 0.0, 0.0]
    (PHCXOperations.py:331-332), before any engine call."""
    ops = profile_ops.PHCXOperations(False)
    assert ops.getSubbandParameters(1) == [0.0, 0.0, 0.0]
    assert ops.getSubbandParameters(0, None, None) == [0.0, 0.0, 0.0]


def test_reference_xmldata_is_accepted(tmp_path):
    """PHCXOperations takes the reference's own xmldata (the minidom Document PHCXFile.load
    keeps, PHCXFile.py:103-104) or its text, at the section the reference passes: the arrays
    are those of the path parser."""
    import gzip
    from xml.dom import minidom

    from pulsarfeatureextractor_amd import phcx
    from test_phcx_native import _write_golden

    path = _write_golden(str(tmp_path), "bates22_phcx128", range(1))[0]
    with gzip.open(path, "rb") as f:
        raw = f.read()
    ref = phcx.parse(path)
    for doc in (minidom.parseString(raw), raw):
        c = profile_ops.PHCXOperations._cand(doc, 1)
        for k in ("profile", "lyon_dm", "subbands", "dm_curve", "scal"):
            assert np.array_equal(getattr(c, k), getattr(ref, k)), k
    with pytest.raises(ValueError):
        profile_ops.PHCXOperations._cand(ref, 0)

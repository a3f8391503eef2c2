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

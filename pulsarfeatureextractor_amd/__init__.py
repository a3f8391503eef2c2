"""pulsarfeatureextractor_amd — MI355X-native batched pulsar-candidate feature engine.

Drop-in for the per-candidate score path of scienceguyrob/PulsarFeatureExtractor: the 8 Lyon
moment features and the 22 Bates scores, computed in batches by gfx950 HIP kernels behind
the C-ABI in include/pfe.h (libpfe.so, bound with ctypes in ``_native``).
"""
__version__ = "0.1.0"

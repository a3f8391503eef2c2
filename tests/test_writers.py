"""Writers reproduce DataProcessor's text (DataProcessor.py:305-447) with Python-2.7 float
str() semantics."""
import math

from pulsarfeatureextractor_amd import writers


def test_py2_str_cases():
    # values of Python 2.7's str(float) (12 significant digits, '.0' for integral values)
    cases = {0.1: "0.1", 1.0 / 3: "0.333333333333", 1e20: "1e+20", 100.0: "100.0",
             -0.0: "-0.0", 123456789.123456789: "123456789.123", 1e-5: "1e-05",
             2.5e-300: "2.5e-300", 12345678901.0: "12345678901.0",
             123456789012.0: "123456789012.0", 1234567890123.0: "1.23456789012e+12",
             5e-324: "4.94065645841e-324", 1e16: "1e+16", 0.0001: "0.0001"}
    for v, s in cases.items():
        assert writers.py2_str(v) == s, (v, writers.py2_str(v), s)


def test_nan_inf_replacement():
    line = writers.score_line("a/b.phcx.gz", [float("nan"), math.inf, -math.inf, 1.5])
    assert line == "a/b.phcx.gz,0,0,-0,1.5"
    assert writers.arff_line("c", [1.0, float("nan")]) == "1.0,0,?%c"
    assert writers.dat_text([2.0, math.inf]) == "2.0,0"


def test_arff_headers():
    h = writers.arff_header("scores", 22)
    assert h.count("@attribute Score") == 22 and h.endswith("@attribute class {0,1}\n@data\n")
    d = writers.arff_header("dmprof")
    assert "@attribute DM_kurtosis numeric\n" in d and d.count("@attribute") == 9


def _edge_values(rng, n):
    import numpy as np

    v = rng.standard_normal((n, 22)) * 10.0 ** rng.integers(-320, 300, (n, 22))
    special = [0.0, -0.0, float("nan"), -float("nan"), math.inf, -math.inf, 1.0, 100.0,
               1e20, 1e-5, 123456789012.0, 1234567890123.0, 5e-324, 1.7976931348623157e308,
               0.5, 2.5, 1e16, 12345678901.5]
    for i, s in enumerate(special):
        v[i % n, i % 22] = s
    v[n // 2] = np.round(v[n // 2])          # integral values get ".0"
    return v


def test_native_formatter_matches_python_writers():
    """pfe_format_rows (the batched product path's writer) == score_line / arff_line /
    dat_text, including names with 'nan'/'inf' in them, for every row."""
    import numpy as np

    from pulsarfeatureextractor_amd import _native

    rng = np.random.default_rng(5)
    n = 3000
    vals = _edge_values(rng, n)
    names = [f"/d/fi{'nan' if i % 7 == 0 else ''}cial/cand_{i}inf{'nanan' if i % 5 == 0 else ''}.phcx.gz"
             for i in range(n)]
    skip = (rng.random(n) < 0.1).astype(np.uint8)
    keep = [i for i in range(n) if not skip[i]]
    got = _native.format_rows(names, vals, 0, skip).decode()
    assert got == "".join(writers.score_line(names[i], vals[i]) + "\n" for i in keep)
    got = _native.format_rows(names, vals, 1, skip, threads=3).decode()
    assert got == "".join(writers.arff_line(names[i], vals[i]) + "\n" for i in keep)
    got = _native.format_rows(names, vals[:, :8], 2).decode()
    assert got == "".join(writers.dat_text(vals[i, :8]) + "\n" for i in range(n))
    assert _native.format_rows([], np.zeros((0, 22))) == b""

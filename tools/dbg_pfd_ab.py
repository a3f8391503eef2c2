import os, sys, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
from test_oracle_pfd import build_files, load_set
from pulsarfeatureextractor_amd import pfd
from pulsarfeatureextractor_amd._native import Engine
import tempfile
g = load_set("pfd_64x16")
d = tempfile.mkdtemp()
files = build_files(d, g)
datas = [pfd.read(f) for f in files]
profs, subfreqs, scal = pfd.batch_inputs(datas)
print("shape", profs.shape)
res = {}
for v in ("1", "0"):
    os.environ["PFE_PFD4"] = v
    with Engine(0) as e:
        res[v] = e.pfd_dmprof(profs, subfreqs, scal)
a, b = res["1"]["chis"], res["0"]["chis"]
bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
print("rows with diffs", np.where(bad.any(1))[0][:10])
print("k with diffs (row 1)", np.where(bad[1])[0])
print(a[1][:12]); print(b[1][:12])
print("profile equal", np.array_equal(res["1"]["profile"], res["0"]["profile"]))

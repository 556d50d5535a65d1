"""debug: poly_poly contact operator of a given library vs the golden fixture."""
import os
import sys

import numpy as np

lib = sys.argv[1]
os.environ["COTIX_AMD_LIB"] = os.path.abspath(lib)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import parallax_amd as pa  # noqa: E402
g = np.load(os.path.join(ROOT, "tests", "golden", "contacts.npz"))
for name in ("poly_poly", "aabb_poly", "circle_poly"):
    a = torch.tensor(g[name + "_a"], device="cuda")
    b = torch.tensor(g[name + "_b"], device="cuda")
    info, err = pa.run_contacts(int(g[name + "_fn"]), a, b)
    got = torch.cat([info.penetration_vector, info.contact_point], 1).cpu().numpy()
    want = g[name + "_out"]
    bad = ~((np.isnan(got) & np.isnan(want)) | (got.view(np.uint32) == want.view(np.uint32)))
    rows = np.unique(np.argwhere(bad)[:, 0])
    print(lib, name, "bad rows", len(rows), "of", len(got), rows[:8])

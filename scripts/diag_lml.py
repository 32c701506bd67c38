"""Diagnose the device LML batch vs the host fp64 objective on one problem."""
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from polyaxon_amd.polytune.bo import HipGP, kernel_np  # noqa: E402

n, d = 200, 16
rng = np.random.RandomState(n + d)
X = rng.uniform(-2, 2, size=(n, d))
y = -np.sum((X - 0.3) ** 2, axis=1) + 0.05 * rng.randn(n)
g = HipGP("cuda")
lls = [math.log(v) for v in (1.5, 2.0, 2.5, 3.0, 3.2, 4.0)]
dev = g.lml_batch(X, y, "rbf", 1.5, lls)
Xd = torch.as_tensor(X, device="cuda")
inv = torch.tensor([math.exp(-2 * l) for l in lls], dtype=torch.float64, device="cuda")
K = torch.empty((len(lls), n, n), dtype=torch.float64, device="cuda")
g.lib.plx_gp_kmat_batch_f64(Xd.data_ptr(), n, d, inv.data_ptr(), len(lls), K.data_ptr(), 0, 1.5, 0.0, 1e-10,
                            g._stream())
torch.cuda.synchronize()
for i, l in enumerate(lls):
    Kh = kernel_np(X, X, "rbf", math.exp(l), 1.5) + 1e-10 * np.eye(n)
    err = float(np.abs(K[i].cpu().numpy() - Kh).max())
    _, info_dev = torch.linalg.cholesky_ex(K[i])
    _, info_h = torch.linalg.cholesky_ex(torch.as_tensor(Kh, device="cuda"))
    try:
        np.linalg.cholesky(Kh)
        hok = True
    except np.linalg.LinAlgError:
        hok = False
    _, info_cpu = torch.linalg.cholesky_ex(torch.as_tensor(Kh))
    print(f"ls={math.exp(l):.2f} dev_lml={dev[i]:.1f} maxerr={err:.2e} info_dev={int(info_dev)} "
          f"info_hostK_on_gpu={int(info_h)} info_cpu_torch={int(info_cpu)} numpy_ok={hok} "
          f"min_eig={float(np.linalg.eigvalsh(Kh)[0]):.3e}")

"""FitOCT.R's batch pipeline on the device (fitoct_amd.pipeline): Courbe.csv
files -> selX -> estimateNoise -> fitMonoExp -> printBr gate -> estimateExpPrior
-> one batched fitExpGP launch (+ the priPost.R prior-predictive launch).
Synthetic data (restated synthData.R); the known answers are the generating
parameters (theta = 1000, 2000, 300 for dataType 2)."""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import prep
from fitoct_amd.pipeline import run_batch
from fitoct_amd.synth import MODULATIONS, synth_decay

pytestmark = pytest.mark.gpu


def test_pipeline_batch_end_to_end(tmp_path):
    data = []
    for i, mod in enumerate(("monoExp",) + MODULATIONS):
        d = synth_decay(481, mod, 40 + i)
        f = tmp_path / mod / "Courbe.csv"
        f.parent.mkdir()
        prep.write_courbe(f, d["x"], d["y"])
        data.append((f"DataSynth_{mod}", str(f)))
    ctrl = {"nb_warmup": 150, "nb_sample": 100, "gridType": "extremal", "Nn": 15,
            "rho_scale": 0, "priorType": "mono"}
    res = run_batch(data, ctrl, nb_chains=4, seed=11, force_gp=True)
    assert [r.tag for r in res] == [t for t, _ in data]
    for r in res:
        assert r.fitGP is not None and r.fitGP_pri is not None
        fit = r.fitGP["fit"]
        assert fit.chains == 4
        th = fit.as_matrix("theta").mean(axis=0)
        np.testing.assert_allclose(th, [1000, 2000, 300], rtol=0.06)
        assert r.fitGP_pri["prior_PD"] == 1
        # prior-predictive theta follows the prior N(theta0, Sigma0) (priPost.R:14)
        thp = r.fitGP_pri["fit"].as_matrix("theta").mean(axis=0)
        np.testing.assert_allclose(thp, r.prior["theta0"], rtol=0.05)
    # FitOCT.R:100 gate: the undisturbed decay passes the mono-exponential Birge test
    assert res[0].br_mono["alert"] is None

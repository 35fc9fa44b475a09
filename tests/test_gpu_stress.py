"""Broad randomized parity on the GPU: 120 small clusters that mix every
encoded feature at once -- resources with overcommitted nodes and pod-count
limits, taints and tolerations, nodeSelector / node affinity incl. Gt/Lt and
matchFields, host ports with specific IPs, required anti-affinity and
affinity on hostname and shared keys (node order, state bits and the domain
path), fallback features -- each plan bit-exact with the oracle (status and
every pod's node of every candidate the device evaluates)."""
import pytest

from randcluster import rand_scenario
from test_gpu_parity import run_scenario

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(120))
def test_gpu_mixed_features(checker, seed):
    shared = seed % 3 == 0
    nodes, spot_pods, cands = rand_scenario(9100 + seed, n_spot=6 + seed % 17, n_cand=8, max_pods=2 + seed % 11,
                                            features=seed % 4 != 3, fallback=seed % 5 == 0,
                                            anti=0.1 + 0.05 * (seed % 6), aff=0.05 * (seed % 7),
                                            shared_keys=shared, valid_selectors=seed % 8 != 7)
    run_scenario(checker, nodes, spot_pods, cands)

"""CPU pin of oracle/gru_torch.py: its functional GRU sequence equals the package's
RecurrentActorCriticNetwork (nn.GRU cell stepped per t with hidden resets -- the intended semantics
of reference recurrent_ppo.py:41-91,94-149) on the same parameters, in float64."""
import numpy as np
import torch

from diamond.recurrent_ppo import RecurrentActorCriticNetwork, RecurrentPPOConfig
from oracle import gru_torch as GT


class Box:
    def __init__(self, n):
        self.shape = (n,)


class Discrete:
    def __init__(self, n):
        self.n = n


def test_oracle_sequence_matches_module():
    T, Nn, D, A = 12, 9, 5, 3
    torch.manual_seed(1)
    net = RecurrentActorCriticNetwork(Box(D), Discrete(A), RecurrentPPOConfig()).double()
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.standard_normal((T, Nn, D)))
    dones = torch.from_numpy(rng.random((T, Nn)) < 0.2)
    hx = torch.from_numpy(rng.standard_normal((1, Nn, 16)))
    with torch.no_grad():
        lg, v, _ = net.get_logits_values_and_hx(obs, hx, dones)
    p = {n: t.detach() for n, t in net.named_parameters()}
    assert list(p) == GT.GRU_NAMES
    lg2, v2 = GT.sequence(p, obs, dones, hx[0])
    torch.testing.assert_close(lg2, lg, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(v2, v, rtol=1e-12, atol=1e-12)

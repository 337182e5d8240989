"""GPU: the agent forward's short-unroll variant (t2o_agent.hip agent_fwd_kernel LOOP:
unrolls of <= 4 steps launch only the resident workgroups and loop each wave over
16-row tiles) against the one-tile-per-wave kernel a longer unroll runs, on a batch
with several tiles per wave (4096 episodes x 16 agents = 4096 tiles): the first
steps' Q and hidden rows must be bit-identical, fp32 and bf16."""
import dataclasses

import pytest
import torch

from tests.gpu_util import require_gpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("A,B", [(16, 4096), (8, 6000)])
def test_short_unroll_tile_loop_matches_long_unroll(prec, A, B):
    require_gpu()
    from t2omca_amd import ops
    from t2omca_amd.modules import TransformerAgent
    from t2omca_amd.synthetic import make_args
    torch.manual_seed(3)
    agent = TransformerAgent(None, make_args(A)).cuda()
    shape = dataclasses.replace(agent.shape, prec=prec)
    pack = ops.pack_params(shape, torch.cat([p.detach().reshape(-1) for p in agent.parameters()]))
    g = torch.Generator(device="cuda").manual_seed(7)
    obs = torch.randn(B, 6, A, 9 * A, device="cuda", generator=g)
    h0 = torch.randn(B * A, shape.E, device="cuda", generator=g)
    q6, h6 = ops.agent_unroll_fwd(shape, pack, obs, h0_on=h0)          # one tile per wave
    for T in (1, 4):                                                   # the tile loop
        qT, hT = ops.agent_unroll_fwd(shape, pack, obs[:, :T], h0_on=h0)
        assert torch.equal(qT, q6[:, :T]) and torch.equal(hT, h6[:, :T]), (prec, A, B, T)

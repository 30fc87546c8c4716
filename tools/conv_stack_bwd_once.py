"""A few fused conv-stack backward launches at 1024 frames (C4-chunk shape class) for PMC
passes (tools/README: rocprofv3 --pmc ... -- python tools/conv_stack_bwd_once.py)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd.layers import LayerExecutor
    from xagents_amd.nets import Adam, ModelReader
    dev = torch.device('cuda')
    cfg = ROOT / 'xagents_amd' / 'dqn' / 'models' / 'cnn.cfg'
    model = ModelReader(str(cfg), [6], (84, 84, 1), Adam(), seed=1, device=dev).build_model()
    B = 1024
    ex = LayerExecutor(model, B)
    x = torch.randint(0, 256, (B, 84, 84, 1), dtype=torch.uint8, device=dev)
    ex.forward(x)
    d = torch.randn(B, 6, device=dev)
    g = torch.zeros(model.n_params, device=dev)
    for _ in range(3):
        ex.backward([d], g)
    torch.cuda.synchronize()
    print('ok')


if __name__ == '__main__':
    main()

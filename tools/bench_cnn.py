"""Time the CNN (dqn/models/cnn.cfg) forward / backward on the layer executor."""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd.layers import LayerExecutor
    from xagents_amd.nets import Adam, ModelReader
    dev = torch.device('cuda')
    m = ModelReader(str(ROOT / 'xagents_amd/dqn/models/cnn.cfg'), [6], (84, 84, 1), Adam(),
                    seed=5, device=dev).build_model()
    for B in (32, 64, 128):
        ex = LayerExecutor(m, B)
        x = torch.randint(0, 256, (B, 84, 84, 1), dtype=torch.uint8, device=dev)
        d = torch.randn(B, 6, device=dev)
        g = torch.zeros(m.n_params, device=dev)
        for _ in range(3):
            ex.forward(x)
            ex.backward([d], g)
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        n = 10
        e[0].record()
        for _ in range(n):
            ex.forward(x)
        e[1].record()
        for _ in range(n):
            ex.backward([d], g)
        e[2].record()
        torch.cuda.synchronize()
        f = e[0].elapsed_time(e[1]) / n
        b = e[1].elapsed_time(e[2]) / n
        gfl = 66.24e6 * B
        print(f'B={B}: forward {f*1e3:.1f} us ({gfl/f/1e9:.1f} TFLOP/s), backward {b*1e3:.1f} us '
              f'({2*gfl/b/1e9:.1f} TFLOP/s)', flush=True)


if __name__ == '__main__':
    main()

"""Per-phase shader-clock stamps of the fused conv-stack backward (diagnostic build:
python tools/build_variant.py cstamp -DXA_STAMPS --src conv_stack): block 0 wave 0's cycles
in staging, (a) dW3, (b) dZ2, (c) dW2, (d) dZ1, (e) dW1 (each up to the barrier that ends it;
the phases' work is split over 8 waves, wave 0's share is stamped)
and the partial write, summed over the launch's groups, averaged over launches.
usage: XA_LIB=tools/diag_lib/libxa_cstamp.so python tools/conv_stack_stamps.py [frames ...]"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    from xagents_amd import _lib
    from xagents_amd.layers import LayerExecutor
    from xagents_amd.nets import Adam, ModelReader
    lib = _lib.load(os.environ['XA_LIB'])
    _lib._lib = lib
    dev = torch.device('cuda')
    cfg = ROOT / 'xagents_amd' / 'dqn' / 'models' / 'cnn.cfg'
    names = ['stage', '(a) dW3', '(b) dZ2', '(c) dW2', '(d) dZ1', '(e) dW1', 'partials', 'entry']
    for B in [int(a) for a in sys.argv[1:]] or [64, 1024]:
        model = ModelReader(str(cfg), [6], (84, 84, 1), Adam(), seed=1, device=dev).build_model()
        ex = LayerExecutor(model, B)
        x = torch.randint(0, 256, (B, 84, 84, 1), dtype=torch.uint8, device=dev)
        ex.forward(x)
        d = torch.randn(B, 6, device=dev)
        g = torch.zeros(model.n_params, device=dev)
        buf = (ctypes.c_ulonglong * 64)()
        for _ in range(3):
            ex.backward([d], g)
        torch.cuda.synchronize()
        lib.xa_diag_read_stamps_conv(buf)  # reset
        n = 10
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(n):
            ex.backward([d], g)
        ev[1].record()
        torch.cuda.synchronize()
        lib.xa_diag_read_stamps_conv(buf)
        st = np.array(buf[:8], np.float64) / n
        tot = st.sum()
        groups = -(-(B * 84) // 16)
        per_wg = -(-groups // 256)
        print(f'frames {B}: {groups} groups, <= {per_wg} per workgroup; backward (+ dense) '
              f'{ev[0].elapsed_time(ev[1]) / n * 1e3:.1f} us per call')
        for i, nm in enumerate(names):
            print(f'  {nm:10s} {st[i]:10.0f} cyc {100 * st[i] / tot:5.1f} %  '
                  f'{st[i] / per_wg:9.0f} cyc per group')


if __name__ == '__main__':
    main()

"""Host cost of a per-step D2H statistics copy into pinned memory (copy_ call time), by
stream (side / launch) and pinned-allocation form; prints the calls slower than 1 ms."""
import time


def trial(side_stream, alloc, steps=80):
    import torch
    dev = 'cuda'
    pack = torch.zeros(16 * 129 + 16 * 128 + 200, device=dev)
    if alloc == 'pin_memory()':
        hosts = [torch.zeros(pack.shape).pin_memory() for _ in range(2)]
    else:
        hosts = [torch.empty(pack.shape, pin_memory=True) for _ in range(2)]
    evs = [torch.cuda.Event(), torch.cuda.Event()]
    roll = torch.cuda.Event()
    side = torch.cuda.Stream(device=dev) if side_stream else torch.cuda.current_stream()
    slow = []
    for k in range(steps):
        torch.cuda._sleep(300_000)
        roll.record()
        side.wait_event(roll)
        t = time.perf_counter()
        with torch.cuda.stream(side):
            hosts[k % 2].copy_(pack, non_blocking=True)
            evs[k % 2].record()
        d = time.perf_counter() - t
        if d > 1e-3:
            slow.append((k, round(d * 1e3, 2)))
        if k:
            evs[(k - 1) % 2].synchronize()
    torch.cuda.synchronize()
    return slow


def main():
    for side in (True, False):
        for alloc in ('pin_memory()', 'empty(pin_memory=True)'):
            print(f'side={side} alloc={alloc}: slow copy_ calls {trial(side, alloc)}')
    print(f'again side=True pin_memory(): {trial(True, "pin_memory()")}')


if __name__ == '__main__':
    main()

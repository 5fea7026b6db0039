"""Per-launch cost of back-to-back kernels in a HIP-graph replay (tools only): N launches of a one-element add, of
an add over 4 MB and over 32 MB, captured and replayed; prints microseconds per launch (wall time of the replay
÷ N) so the fixed boundary cost of a launch in the c3 step can be read off.

    python tools/launch_probe.py [--n 256] [--reps 20]
"""
import argparse

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda"
    for label, numel in (("1 element", 1), ("4 MB", 1 << 20), ("32 MB", 1 << 23)):
        x = torch.zeros(numel, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            x.add_(1.0)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(args.n):
                    x.add_(1.0)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (args.reps * args.n)
        print(f"{label:10s}: {us:7.2f} us per launch in a graph of {args.n} (bytes moved per launch "
              f"{8 * numel / 1e6:.1f} MB -> {8 * numel / (us * 1e-6) / 1e12:.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()

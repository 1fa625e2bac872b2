#!/usr/bin/env python3
"""Do independent branches of one replayed hipGraph run concurrently on this ROCm?  Two chains of
K small dependent kernels captured on two forked streams vs one chain: replay times."""
import torch

K = 60


def chain(x, k):
    for _ in range(k):
        x.mul_(1.0001).add_(0.5)


def timed(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    dev = torch.device("cuda")
    a = torch.zeros(1 << 16, device=dev)
    b = torch.zeros(1 << 16, device=dev)
    cur = torch.cuda.current_stream()
    for prio in (0, -1):
        s1, s2 = torch.cuda.Stream(priority=prio), torch.cuda.Stream(priority=prio)
        # one chain
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            chain(a, K)
        # two chains on forked streams
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            s1.wait_stream(torch.cuda.current_stream())
            s2.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s1):
                chain(a, K)
            with torch.cuda.stream(s2):
                chain(b, K)
            torch.cuda.current_stream().wait_stream(s1)
            torch.cuda.current_stream().wait_stream(s2)
        # the same two chains, serial on one stream
        g3 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g3):
            chain(a, K)
            chain(b, K)
        t1, t2, t3 = timed(g1), timed(g2), timed(g3)
        print(f"priority {prio}: one chain {t1:7.1f} us | two forked chains {t2:7.1f} us | two serial {t3:7.1f} us",
              flush=True)
        # two single-chain graphs replayed on two streams (one graph per lane, joined by events)
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga):
            chain(a, K)
        with torch.cuda.graph(gb):
            chain(b, K)

        def two_graphs(reps=20):
            c = torch.cuda.current_stream()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                s1.wait_stream(c)
                s2.wait_stream(c)
                with torch.cuda.stream(s1):
                    ga.replay()
                with torch.cuda.stream(s2):
                    gb.replay()
                c.wait_stream(s1)
                c.wait_stream(s2)
            e.record()
            e.synchronize()
            return s.elapsed_time(e) * 1e3 / reps

        two_graphs(3)
        t4 = two_graphs()

        def eager(reps=5):
            c = torch.cuda.current_stream()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                s1.wait_stream(c)
                s2.wait_stream(c)
                with torch.cuda.stream(s1):
                    chain(a, K)
                with torch.cuda.stream(s2):
                    chain(b, K)
                c.wait_stream(s1)
                c.wait_stream(s2)
            e.record()
            e.synchronize()
            return s.elapsed_time(e) * 1e3 / reps

        eager(2)
        t5 = eager()
        print(f"priority {prio}: two graphs on two streams {t4:7.1f} us | eager two streams {t5:7.1f} us", flush=True)
    del cur


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Do two hipGraphs replayed on two streams overlap?  Spin kernels (torch.cuda._sleep: one
thread, fixed cycles) so that overlap shows as wall ~ max instead of sum: eager on two streams,
one graph with two forked branches, two single-chain graphs on two streams."""
import time

import torch

CYC = 2_000_000   # ~1 ms at ~2 GHz
K = 4


def chain():
    for _ in range(K):
        torch.cuda._sleep(CYC)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cur = torch.cuda.current_stream()

    def one():
        chain()

    def eager2():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            chain()
        with torch.cuda.stream(s2):
            chain()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        chain()
    gf = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf):
        c = torch.cuda.current_stream()
        s1.wait_stream(c)
        s2.wait_stream(c)
        with torch.cuda.stream(s1):
            chain()
        with torch.cuda.stream(s2):
            chain()
        c.wait_stream(s1)
        c.wait_stream(s2)
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga):
        chain()
    with torch.cuda.graph(gb):
        chain()

    def graphs2():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def graph_and_eager():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            chain()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    print(f"one chain eager        {timed(one):7.2f} ms", flush=True)
    print(f"one chain graph        {timed(g1.replay):7.2f} ms", flush=True)
    print(f"two chains eager       {timed(eager2):7.2f} ms  (overlap -> ~one chain)", flush=True)
    print(f"one graph, 2 branches  {timed(gf.replay):7.2f} ms", flush=True)
    print(f"two graphs, 2 streams  {timed(graphs2):7.2f} ms", flush=True)
    print(f"graph + eager          {timed(graph_and_eager):7.2f} ms", flush=True)


if __name__ == "__main__":
    main()

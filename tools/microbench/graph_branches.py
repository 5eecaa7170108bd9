"""Do the parallel branches of one captured HIP graph run concurrently?

A graph with two independent spin kernels forked onto a side stream and
joined, against the same two kernels in series, and against two separate
graphs replayed on two streams.  Prints one JSON line (µs per replay).
Usage (GPU box): python tools/microbench/graph_branches.py"""
import json

import torch


def spin(cycles):
    torch.cuda._sleep(cycles)


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1000.0 * a.elapsed_time(b) / reps


def main():
    torch.cuda.init()
    cyc = 100000  # ~40-50 µs at the shader clock
    main_s = torch.cuda.Stream()
    side = torch.cuda.Stream()
    one = torch.cuda.CUDAGraph()
    with torch.cuda.graph(one, stream=main_s):
        spin(cyc)
    serial = torch.cuda.CUDAGraph()
    with torch.cuda.graph(serial, stream=main_s):
        spin(cyc)
        spin(cyc)
    forked = torch.cuda.CUDAGraph()
    with torch.cuda.graph(forked, stream=main_s):
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            spin(cyc)
        spin(cyc)
        main_s.wait_stream(side)
    side_g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(side_g, stream=side):
        spin(cyc)
    res = {}
    with torch.cuda.stream(main_s):
        res["one_us"] = timed(one.replay)
        res["serial_us"] = timed(serial.replay)
        res["forked_us"] = timed(forked.replay)

        def two_graphs():
            side.wait_stream(main_s)
            one.replay()
            with torch.cuda.stream(side):
                side_g.replay()
            main_s.wait_stream(side)
        res["two_graphs_two_streams_us"] = timed(two_graphs)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

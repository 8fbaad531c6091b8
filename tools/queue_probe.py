"""Hardware-queue map of a pipeline rank's streams on one GPU (parallel/queues.py probe).

    python tools/queue_probe.py [--out profiles/r3_queue_probe.json] [--timeout-us 20000]

Creates the stream set a PP>1 rank drives, in the runtime's creation order -- the torch
compute stream, the process-wide comm stream slots of csrc/comm/rccl_engine.h (fwd p2p,
bwd p2p, collectives; created when the pipeline engine is built, before the first step),
the dW side stream of models/native.py (first backward), two microbatch-lane streams
(PP=1 only) and torch pool streams of both priorities (what ProcessGroupNCCL and graph
capture draw from) -- then probes every pair with the bounded spin/flag kernel pair
(csrc/kernels/probe.hip) and a captured graph forking onto the dW side stream against each
comm stream.  A pair is "shared" when the flag store could not run while the spinner was
resident.  The JSON records the matrix and the conclusion the runtime draws
(PipelineRuntime._prove): whether every comm stream has a queue of its own.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--timeout-us", type=int, default=20000)
    a = ap.parse_args()
    import torch
    import mipipe  # noqa: F401
    from mipipe.parallel.queues import comm_streams, rank_streams, shares_queue
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    env = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")}
    streams = {"compute": int(torch.cuda.current_stream(dev).cuda_stream)}
    streams.update(comm_streams(dev))                       # engine built at trainer init
    rs = rank_streams(dev)                                  # dW side stream (first backward)
    streams["dw_side"] = rs["dw_side"]
    for i in range(2):
        streams[f"lane{i + 1}"] = int(torch.cuda.Stream(device=dev).cuda_stream)
    for i in range(2):
        streams[f"pool_normal{i}"] = int(torch.cuda.Stream(device=dev, priority=0).cuda_stream)
        streams[f"pool_high{i}"] = int(torch.cuda.Stream(device=dev, priority=-1).cuda_stream)
    names = list(streams)
    pairs = {}
    shared = []
    for i, x in enumerate(names):
        for y in names[i + 1:]:
            sh, us = shares_queue(streams[x], streams[y], dev, a.timeout_us)
            pairs[f"{x}|{y}"] = {"shared": sh, "wait_us": round(us, 1)}
            if sh:
                shared.append(f"{x}|{y}")
    graph_pairs = {}
    for c in ("comm:fwd", "comm:bwd", "comm:coll"):
        for role in ("setter", "waiter"):
            if role == "setter":   # comm spins, the graph's forked dW branch stores the flag
                sh, us = shares_queue(streams[c], streams["dw_side"], dev, a.timeout_us, graph="setter")
            else:                  # the graph's forked branch spins, the comm stream stores
                sh, us = shares_queue(streams["dw_side"], streams[c], dev, a.timeout_us, graph="waiter")
            graph_pairs[f"{c}|graph(dw_side branch as {role})"] = {"shared": sh, "wait_us": round(us, 1)}
            if sh:
                shared.append(f"{c}|graph:{role}")
    comm = [n for n in names if n.startswith("comm:")]
    comm_shared = [p for p in shared if any(p.startswith(c + "|") or ("|" + c) in p for c in comm)
                   and not any(("pool_" in p, "lane" in p))]
    out = {
        "device": torch.cuda.get_device_name(dev),
        "env": env,
        "streams_in_creation_order": names,
        "pairs": pairs,
        "graph_pairs": graph_pairs,
        "shared_pairs": shared,
        "comm_streams_independent_of_rank_streams": not comm_shared,
        "runtime_conclusion": ("collectives overlap the flush (the default MIPIPE_COLL_OVERLAP=probe admits it)"
                               if not comm_shared else
                               "comm streams share queues: collectives deferred to the step end (serial model)"),
        "note": ("PipelineRuntime._prove runs this probe per rank and MIN-votes the verdict over the world; "
                 "microbatch lanes at PP > 1 are accepted only on streams with queues apart from compute "
                 "and every comm stream"),
    }
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()

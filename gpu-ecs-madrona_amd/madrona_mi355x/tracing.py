"""Device-trace analysis (the per-step reading scripts/parse_device_tracing.py
does of the same 40-byte records, reference parse_device_logs /
serialized_analysis, scripts/parse_device_tracing.py:11-143).

split_steps(records) -> list of per-step record arrays (a step opens with a
calibration record whose logIndex is 0);
node_spans(step) -> {nodeID: (funcID, numInvocations, start_ns, end_ns)};
block_spans(step) -> {(smID, numInvocations, nodeID, blockID): (start, end)};
summarize(records, func_names) -> per node kind: launches per step and mean
ns per step, over every complete step.
"""
import numpy as np

CALIBRATION, NODE_START, NODE_FINISH, BLOCK_START, BLOCK_WAIT, BLOCK_EXIT = range(6)


def split_steps(records):
    starts = np.nonzero((records["event"] == CALIBRATION) & (records["logIndex"] == 0))[0]
    bounds = list(starts) + [len(records)]
    return [records[bounds[i]:bounds[i + 1]] for i in range(len(starts))]


def node_spans(step):
    spans = {}
    for r in step[(step["event"] == NODE_START) | (step["event"] == NODE_FINISH)]:
        n = int(r["nodeID"])
        f, inv, s, e = spans.get(n, (int(r["funcID"]), int(r["numInvocations"]), None, None))
        if (f, inv) != (int(r["funcID"]), int(r["numInvocations"])):
            raise ValueError(f"node {n}: start / finish disagree on (funcID, numInvocations)")
        if r["event"] == NODE_START:
            if s is not None:
                raise ValueError(f"node {n}: two starts")
            s = int(r["cycleCount"])
        else:
            if e is not None:
                raise ValueError(f"node {n}: two finishes")
            e = int(r["cycleCount"])
        spans[n] = (f, inv, s, e)
    return spans


def block_spans(step):
    spans = {}
    for r in step[(step["event"] == BLOCK_START) | (step["event"] == BLOCK_WAIT)]:
        key = (int(r["smID"]), int(r["numInvocations"]), int(r["nodeID"]), int(r["blockID"]))
        s, e = spans.get(key, (None, None))
        if r["event"] == BLOCK_START:
            if s is not None:
                raise ValueError(f"block {key}: two starts in one step")
            s = int(r["cycleCount"])
        else:
            if e is not None:
                raise ValueError(f"block {key}: two waits in one step")
            e = int(r["cycleCount"])
        spans[key] = (s, e)
    return spans


def summarize(records, func_names):
    steps = [s for s in split_steps(records) if np.any(s["event"] == BLOCK_EXIT)]
    out = {}
    for st in steps:
        for n, (f, _, s, e) in node_spans(st).items():
            name = func_names[f] if f < len(func_names) else str(f)
            d = out.setdefault(name, {"launches": 0, "ns": 0})
            d["launches"] += 1
            d["ns"] += e - s
    for d in out.values():
        d["launches_per_step"] = d["launches"] / max(1, len(steps))
        d["ns_per_step"] = d["ns"] / max(1, len(steps))
    return out


def check_contract(records, func_names, num_invocations, block_records):
    """Raises AssertionError unless the records are what
    scripts/parse_device_tracing.py accepts (parse_device_logs /
    block_analysis, :11-118, :146-230): each step opens with a calibration
    record (logIndex 0) and has one blockExit; nodes have one start and one
    finish, numbered 0..n-1 in stream order, spans serial; with block
    records, one blockStart / blockWait pair per (SM, launch, node, block)
    key inside its node's span.  Returns the number of steps."""
    steps = split_steps(records)
    assert steps, "no calibration record"
    for st in steps:
        assert st[0]["event"] == CALIBRATION and st[0]["logIndex"] == 0
        assert (st["logIndex"][1:] > 0).all()
        assert (st["event"] == BLOCK_EXIT).sum() == 1
        nodes = node_spans(st)
        ids = sorted(nodes)
        assert ids == list(range(len(ids))), ids
        for i in ids:
            f, inv, s, e = nodes[i]
            assert s is not None and e is not None and s <= e, i
            assert f < len(func_names) and inv == num_invocations
        for a, b in zip(ids, ids[1:]):
            assert nodes[a][3] <= nodes[b][2], (a, b)
        blocks = block_spans(st)
        if not block_records:
            assert not blocks
            continue
        assert len(blocks) > len(ids)
        for (sm, inv, node, blk), (s, e) in blocks.items():
            assert s is not None and e is not None and s <= e
            _, _, ns, ne = nodes[node]
            assert ns <= s and e <= ne, (node, func_names[nodes[node][0]])
    return len(steps)

"""A HIP graph of the whole encode step.

Round 3 recorded that back-to-back replays of a captured encode step left the GPU in a memory-fault state.
What a captured launch references must outlive every replay: the fused encoder keeps its codebooks, candidate
lists and assign workspace; every per-call tensor of ``RQEncoder.encode`` (the output, level-1 denominators,
global ids, bucket offsets / row permutation / scratch) is allocated inside ``torch.cuda.graph``, i.e. from
the graph's private memory pool, which torch keeps reserved for the graph (a raw stream capture would hand
those blocks back to the caching allocator after capture, and a replay would write freed memory).  The
encode path has no host synchronisation to capture (single_segment and bucket are device-side; the penalty
and group-range checks only sync when the codebooks can need them, never for these shapes)."""
import numpy as np
import pytest
import torch

from generative_ranking_recommender_amd import synth
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN, RQEncoder

pytestmark = pytest.mark.gpu


def test_encode_step_graph_replays_equal_eager():
    dev = torch.device("cuda", 0)
    cb = synth.encode_codebooks(seed=99)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = torch.from_numpy(synth.mixture_rows(0, 200_000)).to(dev)
    eager = enc.encode(x).clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            enc.encode(x)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = enc.encode(x)
    g.replay()
    torch.cuda.synchronize()
    first = out.clone()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(first, eager)
    assert torch.equal(out, eager)
    # the captured step reads x in place: new rows in the same buffer give their own eager IDs
    x.copy_(torch.from_numpy(synth.mixture_rows(200_000, 400_000)).to(dev))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, enc.encode(x))
    del g


def test_encode_list_writes_stay_in_bounds():
    """Every write of the captured encode step whose index comes from a device counter -- rqsid_assign's
    sentinel compaction and the fp32 re-screen's overflow list (csrc/assign_common.h kErrSlot), rqsid_bucket's
    row_index scatter (csrc/rqsid.hip bucket_put) -- is bounded by its slot and raises a bit of a sticky error
    word instead of writing past it.  PROD codebooks, every level, eager and three back-to-back graph
    replays: every word stays 0 (the encoder's assign workspace and both of its bucket workspaces)."""
    dev = torch.device("cuda", 0)
    cb = synth.encode_codebooks(seed=99)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [128, 128, 256],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = torch.from_numpy(synth.mixture_rows(0, 100_000)).to(dev)
    eager = enc.encode(x).clone()
    assert enc._ws.error() == 0
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        enc.encode(x)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = enc.encode(x)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
    assert enc._ws.error() == 0
    words = enc.error_words()
    assert len(words) == 3 and all(int(w.item()) == 0 for w in words)  # assign + the two levels' buckets
    del g


def test_encode_raises_on_a_set_error_word():
    """a dropped counter-driven write must not pass silently.  RQEncoder.encode reads the error
    words after the call (one host sync) and raises; here a bucket word is set by hand."""
    dev = torch.device("cuda", 0)
    cb = synth.encode_codebooks(seed=5, need=(16, 16, 32), n_cand=320, pool_rows=8192)
    enc = RQEncoder([torch.from_numpy(cb[k]) for k in ("c0", "c1", "c2")], [16, 16, 32],
                    match=torch.from_numpy(cb["match"]), semantics=HIERARCHICAL_TRAIN, device=dev)
    x = torch.from_numpy(synth.mixture_rows(0, 4096)).to(dev)
    enc.encode(x)
    enc.error_words()[-1].fill_(1)
    with pytest.raises(RuntimeError, match="error word"):
        enc.encode(x)

"""The trainer's graph set (trainer.py): one captured graph per epoch of full batches, up to
MAX_GRAPH_STEPS steps, a longer epoch's remainder as one more graph; graph_replays covers any
count with the captured sizes, largest first."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))

import trainer as T  # noqa: E402


@pytest.mark.parametrize("full", [1, 2, 7, 20, 32, 33, 511, 512, 513, 600, 1024, 1300])
def test_epoch_graph_sizes_cover_the_epoch(full):
    sizes = T.epoch_graph_sizes(full)
    reps = T.graph_replays(full, tuple(sizes))
    assert sum(reps) == full
    assert reps[0] == min(full, T.MAX_GRAPH_STEPS)
    assert reps.count(reps[0]) == full // reps[0]  # whole-epoch graphs first
    assert len(reps) - full // reps[0] <= 1  # the remainder: one graph
    assert set(reps) <= set(sizes)


def test_graph_replays_any_order_of_sizes():
    assert T.graph_replays(20, (1, 2, 4, 8, 32)) == [8, 8, 4]
    assert T.graph_replays(20, (20, 8, 4, 2, 1)) == [20]
    assert T.graph_replays(0, (8, 1)) == []

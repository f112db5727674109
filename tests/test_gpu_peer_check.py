"""The xGMI peer check of the GPU probe (devspace_amd/gpucheck.py peer_check), on a fake probe:
which pairs it reports (no GPU needed; the HIP side is tests/test_gpucheck.py)."""
from devspace_amd import gpucheck


class FakeProbe:
    def __init__(self, rates, no_peer=()):
        self.rates, self.no_peer = rates, set(no_peer)

    def peer_access(self, a, b):
        return 0 if (a, b) in self.no_peer else 1

    def peer_gbps(self, a, b, nbytes=0, iters=0):
        return self.rates.get((a, b), 50.0)


def test_healthy_node_has_no_problems():
    pairs, problems = gpucheck.peer_check(FakeProbe({}), 8)
    assert len(pairs) == 56 and not problems


def test_missing_peer_access_and_a_slow_link_are_reported():
    probe = FakeProbe({(2, 5): 12.0, (3, 1): -1.0}, no_peer=[(6, 7)])
    pairs, problems = gpucheck.peer_check(probe, 8)
    text = "\n".join(problems)
    assert "gpu6 -> gpu7: no peer access" in text
    assert "gpu2 -> gpu5: peer copy 12 GB/s, under half the median pair (50 GB/s)" in text
    assert "gpu3 -> gpu1: peer copy failed" in text
    assert len(problems) == 3, problems

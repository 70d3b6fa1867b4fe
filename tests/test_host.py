"""Host-side logic that needs no GPU: rollout stream seeding, library build staleness."""
import numpy as np


def test_stream_seeds_distinct_and_reproducible():
    """Every rollout call of a SOARM101DataGenerator draws from its own stream (the
    reference's datasets come from one advancing np.random stream, :97-132)."""
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import stream_seed
    s = [stream_seed(42, k) for k in range(4096)]
    assert len(set(s)) == len(s)
    assert all(0 <= x < 2 ** 32 for x in s)
    assert s[:8] == [stream_seed(42, k) for k in range(8)]
    assert set(stream_seed(43, k) for k in range(64)).isdisjoint(s[:64])
    # the reset key only uses the low 32 bits of the seed: the streams' keys differ there
    assert len(set(x & 0xFFFFFFFF for x in s)) == len(s)
    # sine tables drawn from distinct streams differ
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import SineInputGenerator
    a = SineInputGenerator(16, rng=np.random.default_rng(s[0]))
    b = SineInputGenerator(16, rng=np.random.default_rng(s[1]))
    assert not np.allclose(a.freq_table, b.freq_table)

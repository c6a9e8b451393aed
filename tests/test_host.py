

def test_run_adam_signature():
    """utils/training_utils.py:4 drop-in: run_adam(model, num_iter, train_iter, lr, compile=True)."""
    import inspect
    from utils.training_utils import run_adam
    assert list(inspect.signature(run_adam).parameters) == ["model", "num_iter", "train_iter", "lr", "compile"]


def test_dataset_pipeline_semantics():
    """tf.data replacement: shuffle(buffer = all).batch(b).repeat():
    each pass is a fresh permutation, the short remainder batch is emitted, the
    stream is seeded, components stay aligned, device/host arrays both work."""
    import itertools
    import numpy as np
    import torch
    from utils.data import Dataset
    X = np.arange(600, dtype=np.float32)[:, None]
    Y = 10 * np.arange(600, dtype=np.float32)[:, None]
    ds = Dataset.from_tensor_slices((X, Y)).shuffle(buffer_size=600, seed=0).batch(500).repeat()
    it = iter(ds)
    batches = list(itertools.islice(it, 6))
    assert [len(b[0]) for b in batches] == [500, 100] * 3
    for bx, by in batches:
        assert np.array_equal(by, 10 * bx)
    e1 = np.concatenate([b[0][:, 0] for b in batches[:2]])
    e2 = np.concatenate([b[0][:, 0] for b in batches[2:4]])
    assert sorted(e1) == list(range(600)) and sorted(e2) == list(range(600))
    assert not np.array_equal(e1, e2)                      # reshuffled each pass
    again = list(itertools.islice(iter(ds), 2))
    assert np.array_equal(again[0][0], batches[0][0])      # seeded
    assert [len(b[0]) for b in Dataset.from_tensor_slices((X, Y)).batch(500, drop_remainder=True).repeat(2)] == [500, 500]
    # a small shuffle buffer still yields a permutation per pass
    small = list(Dataset.from_tensor_slices(torch.arange(50)).shuffle(8, seed=1).batch(50))
    assert sorted(small[0].tolist()) == list(range(50))


def test_toy_datasets_match_reference_generators():
    """utils/dataset_utils.py (drop-in) reproduces the reference's generators
    bit-for-bit (tests/golden/toy_datasets.npz, made by make_golden.py from the
    reference's own utils/dataset_utils.py:84-166)."""
    import os
    import numpy as np
    from utils import dataset_utils as U
    d = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "toy_datasets.npz")))
    for name in ("load_toy_data_categorical", "load_toy_multimodal_data", "load_toy_2d_data",
                 "load_toy_2d_data_categorical", "load_toy_data_assoc"):
        if name == "load_toy_data_assoc":
            np.random.seed(0)
            out = U.load_toy_data_assoc()
        else:
            out = getattr(U, name)(np.random.default_rng(0))
        for key, got in zip(("N", "X", "Y", "Xtest"), out):
            ref = d[f"{name}_{key}"]
            assert np.array_equal(np.asarray(got), ref), (name, key)
            assert np.asarray(got).dtype == ref.dtype, (name, key)


def test_config_expert_cross_knob():
    """K5 cross-term precision knob (config.expert_cross): 'f16' (default, f16x3) or
    'f8' (f16x8, e4m3 cross terms); anything else is refused."""
    import pytest
    from modulatedgps_amd import config
    old = config.expert_cross()
    try:
        for v in ("f8", "f16"):
            config.set_expert_cross(v)
            assert config.expert_cross() == v
        with pytest.raises(ValueError):
            config.set_expert_cross("bf16")
    finally:
        config.set_expert_cross(old)

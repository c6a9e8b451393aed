

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


def test_config_step_schedule_knob():
    """Launch placement of the Cholesky-independent work relative to K3
    (config.step_schedule, host-side only): every documented schedule is accepted,
    anything else is refused."""
    import pytest
    from modulatedgps_amd import config
    old = config.step_schedule()
    try:
        for v in config.STEP_SCHEDULES:
            config.set_step_schedule(v)
            assert config.step_schedule() == v
        with pytest.raises(ValueError):
            config.set_step_schedule("k1_first")
    finally:
        config.set_step_schedule(old)


def test_host_arrays_feed_the_demo_post_processing():
    """predict_* return HostArray (float64 numpy); the demo's numpy lines
    (demos/demo_tf2.py, reference demo_tf2.py:63-72,98-99) and `.numpy()` work."""
    import numpy as np
    from modulatedgps_amd.models import HostArray
    sy = np.random.default_rng(0).standard_normal((100, 50, 1)).view(HostArray)
    samples_y = np.hstack([sy, sy])
    assert samples_y.shape == (100, 100, 1)
    assert np.mean(samples_y, 0).shape == (100, 1)
    assert np.reshape(samples_y, (100 * 100, -1)).shape == (10000, 1)
    assert isinstance(sy.numpy(), np.ndarray) and sy.numpy().dtype == np.float64


def test_env_config_is_validated():
    """MGP_* environment overrides go through the setters (a bad value raises at import)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import modulatedgps_amd.config as c; print(c.expert_format(), c.expert_planes())"
    ok = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                        env={**os.environ, "MGP_K5_FORMAT": "x6", "MGP_K5_PLANES": "2"})
    assert ok.returncode == 0 and ok.stdout.split() == ["x6", "2"]
    for k, v in (("MGP_K5_FORMAT", "bf8"), ("MGP_K5_PLANES", "4"), ("MGP_K5_CROSS", "x"),
                 ("MGP_CONDITIONAL", "f64"), ("MGP_STEP_SCHEDULE", "late")):
        bad = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                             env={**os.environ, k: v})
        assert bad.returncode != 0 and "ValueError" in bad.stderr, (k, v)


def test_bench_refuses_missing_gpus():
    """`bench.py --gpus N` with fewer than N visible devices exits non-zero (here: none)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "MGP_BENCH_SHARE_GPU")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=root, capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 2 and "device(s) visible" in r.stderr

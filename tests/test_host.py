

def test_run_adam_signature():
    """utils/training_utils.py:4 drop-in: run_adam(model, num_iter, train_iter, lr, compile=True)."""
    import inspect
    from utils.training_utils import run_adam
    assert list(inspect.signature(run_adam).parameters) == ["model", "num_iter", "train_iter", "lr", "compile"]

"""Drop-in for the reference's repo-level ``utils`` package (training loop only)."""

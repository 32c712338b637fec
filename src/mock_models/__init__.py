"""
Mock model backends (CPU, no GPU): the reference's ``FakeModel`` echo model and
``mock_batch_inference`` (`/root/reference/src/mock_models/`). They back
BASELINE config 1 (the plumbing benchmark) and the control-plane tests.
"""

from .fake_model import FakeModel
from .mock_inference import mock_batch_inference

__all__ = ["FakeModel", "mock_batch_inference"]

"""Test configuration: ``gpu`` marker, fast settings, registry hygiene."""

import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and the native library")
    config.addinivalue_line("markers", "slow: long-running integration test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _fast_settings():
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.utils import set_test_settings

    snap = Settings.snapshot()
    set_test_settings()
    yield
    for k, v in snap.items():
        setattr(Settings, k, v)

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
EMU = os.path.join(ROOT, "tests", "emu")
if EMU not in sys.path:
    sys.path.insert(0, EMU)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session", autouse=True)
def _torch_runtime_first(request):
    """GPU runs: torch (plumbing for the device-path tests) bundles its own
    HIP runtime, which must initialise before libdpgpu's runtime claims the
    device -- whichever test file runs first."""
    expr = request.config.getoption("markexpr") or ""
    if "gpu" in expr and "not gpu" not in expr:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield


CLS_FORMS = {"auto": 0, "bv": 1, "list": 2}


@pytest.fixture
def cls_form():
    """cls_form(lib, "bv" | "list" | "auto"): classifier form for the image
    builds of `lib` (dpd_debug_set_classifier_form); reset after the test."""
    used = []

    def set_form(lib, form):
        lib.dpd_debug_set_classifier_form(CLS_FORMS[form])
        used.append(lib)

    yield set_form
    for lib in used:
        lib.dpd_debug_set_classifier_form(0)

"""The driver's smoke() (one small add on cuda:0, bit-exact against the oracle) as a GPU test, so
the -m gpu suite exercises exactly what the driver runs before the bench."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_driver_smoke_entry():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import __graft_entry__ as entry
    entry.smoke()

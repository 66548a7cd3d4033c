"""The driver's round-end smoke check (__graft_entry__.smoke) as a GPU test."""
import pytest

pytestmark = pytest.mark.gpu


def test_graft_entry_smoke():
    import __graft_entry__ as g
    g.smoke()

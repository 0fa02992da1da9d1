"""The driver's smoke() entry point, run inside the GPU suite so a broken smoke path fails `pytest -m gpu`."""
import pytest


@pytest.mark.gpu
def test_graft_entry_smoke(capsys):
    import __graft_entry__
    __graft_entry__.smoke()
    assert "bit-identical to the exact oracle" in capsys.readouterr().out

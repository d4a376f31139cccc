"""The verl-side plug point (dots.rl_amd/verl_adapter.py) against the reference's own decorator / worker /
DataProto code. Skipped where /root/reference is absent (the GPU box); the checks run in
a child process so the reference's import stubs never enter this session (tests/verl_adapter_check.py)."""

import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(not os.path.isdir("/root/reference/verl"), reason="needs the reference checkout")
def test_adapter_matches_reference_dispatch_and_dataproto():
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "verl_adapter_check.py")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip().endswith("OK"), r.stdout


def test_adapter_imports_without_verl():
    from dots.rl_amd import verl_adapter

    assert set(verl_adapter.ACTOR_METHODS) >= {"generate_sequences", "compute_log_prob", "compute_ref_log_prob",
                                               "update_actor"}
    with pytest.raises(AttributeError):
        verl_adapter.NoSuchThing  # noqa: B018

"""CPU: differential parity on fresh random traces (tests/scenarios.py random_scenario): the
clean-room restatement (oracle/relay_model) must equal the REAL reference reflector
(oracle/_ref/ref_harness) byte for byte -- captures, receiver-report trailers and all -- on
inputs neither was tuned on.  Runs where the reference tree is present (this container)."""
import pytest

from scenarios import random_scenario

SEEDS = range(64)


def _run(binary, trace, tmp_path, tag):
    import subprocess
    t, c = tmp_path / f"{tag}.edtr", tmp_path / f"{tag}.edcp"
    t.write_bytes(trace)
    subprocess.run([binary, str(t), str(c)], check=True, stderr=subprocess.DEVNULL)
    return c.read_bytes()


@pytest.mark.parametrize("seed", SEEDS)
def test_restatement_matches_reference_on_random_traces(seed, oracle_bins, tmp_path):
    if oracle_bins["ref"] is None:
        pytest.skip("oracle/_ref/ref_harness not built (reference tree absent)")
    tr = random_scenario(seed)
    trace = tr.to_bytes()
    ref = _run(oracle_bins["ref"], trace, tmp_path, "ref")
    port = _run(oracle_bins["port"], trace, tmp_path, "port")
    # a trace whose only session ended before any player joined has an empty capture
    assert port == ref and (len(ref) > 16 or tr.has_lifecycle)

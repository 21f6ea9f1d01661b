"""Shared pytest setup: markers, import paths for the product package
(p2p-file-system-with-gossip-detect-failure-management_amd/gossipsim) and the
test-only oracle (oracle/)."""
import pathlib
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]
PKG_DIR = REPO / "p2p-file-system-with-gossip-detect-failure-management_amd"
for p in (str(REPO), str(PKG_DIR)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built libgossiphip")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as om
    om.build()
    return om

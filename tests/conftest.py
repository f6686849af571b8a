"""Test configuration: registers the ``gpu`` marker and puts the product
package (uncertainty-model_amd/) and the repo root (oracle/) on sys.path."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'uncertainty-model_amd')
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP path)')


def pytest_sessionstart(session):
    """Build libumamd.so once per session (content-hash staleness): a compile
    error then fails the session with hipcc's own message."""
    from umamd import _build
    if _build.needs_build() and _build.can_build():
        _build.build()

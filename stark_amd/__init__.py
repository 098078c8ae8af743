"""stark_amd -- MI355X-native (gfx950) rebuild of stark's data-parallel hot path.

``from stark_amd import *`` binds the submodule ``stark``, like the reference package
(stark/__init__.py:1), so ``stark.Stark`` / ``stark.consensus_avg`` resolve the same way.
"""
__all__ = ["stark"]

from . import stark  # noqa: E402,F401

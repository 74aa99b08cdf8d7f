"""Build hook: compile the in-tree native libraries before packaging.

``pip install .`` on a ROCm host runs ``myfyp_amd.ops.build`` (hipcc, gfx950) and the host-only
control-plane library (g++), so the wheel carries ``myfyp_amd/_native/*.so``. Without hipcc the
package installs CPU-only (the fused paths then raise on a GPU host instead of silently falling back).
"""

import shutil

from setuptools import setup
from setuptools.command.build_py import build_py


class BuildWithNative(build_py):
    def run(self):
        from myfyp_amd.ops import build as native

        native.build_host()
        if shutil.which("hipcc") or shutil.which("/opt/rocm/bin/hipcc"):
            native.build()
        super().run()


setup(cmdclass={"build_py": BuildWithNative})

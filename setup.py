"""setuptools hook: build the gfx950 native library (jax_raft_amd/_C.so) with
hipcc before packaging, so ``pip install .`` / ``python setup.py build_ext
--inplace`` produce the same in-tree artefact as ``__graft_entry__.build()``."""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        from jax_raft_amd._build import build

        build()
        super().run()


setup(cmdclass={"build_py": BuildNative})

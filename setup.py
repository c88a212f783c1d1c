"""Packaging hook: build the gfx950 extension modules in-tree before packaging
(the same build as ``python -m cloud_amd._build``; CMakeLists.txt is the CMake
alternative)."""
from setuptools import setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        from cloud_amd import _build

        _build.build_all()
        super().run()


setup(cmdclass={"build_py": BuildNative})

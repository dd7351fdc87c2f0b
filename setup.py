"""Package metadata for ``mi355x-dp`` (see pyproject.toml for the build / install notes).

    pip install -e .    # editable: native components build in-tree with `mi355x-build`
"""
from setuptools import find_packages, setup

setup(
    name="mi355x-dp",
    version="0.2.0",
    description=("MI355X-native (gfx950) data-parallel training: hand-written HIP kernels, RCCL/xGMI smddp backend, "
                 "SageMaker-workshop compatible API"),
    long_description=open("README.md").read(),
    long_description_content_type="text/markdown",
    python_requires=">=3.9",
    packages=find_packages(include=["mi355x_dp", "mi355x_dp.*"]),
    package_data={"mi355x_dp": ["_native/*.so", "_native/mi355x_launch", "_compat/*/*.py", "_compat/*/*/*.py",
                                "_compat/*/*/*/*.py", "_compat/*/*/*/*/*.py", "_compat/*.py"]},
    # replaces the reference's notebooks/code/r.txt pin list; torch is the only
    # runtime requirement of the training path
    install_requires=["torch>=2.4", "numpy>=1.21", "pillow>=9"],
    extras_require={"mntd": ["scikit-learn>=1.0"], "test": ["pytest>=7", "pytest-timeout>=2"]},
    entry_points={"console_scripts": ["mi355x-build = mi355x_dp.build:main", "mi355x-launch = mi355x_dp.launch:main"]},
)

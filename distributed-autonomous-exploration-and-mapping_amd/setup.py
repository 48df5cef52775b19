"""ament_python packaging of the ROS side (colcon build in a ROS 2 workspace).
libdm.so is built beforehand (make -C csrc) and shipped inside the dm package."""
from glob import glob

from setuptools import setup

setup(
    name="dm_mapping",
    version="0.2.0",
    packages=["dm"],
    package_data={"dm": ["libdm.so"]},
    data_files=[
        ("share/ament_index/resource_index/packages", ["resource/dm_mapping"]),
        ("share/dm_mapping", ["package.xml"]),
        ("share/dm_mapping/launch", glob("launch/*.launch.py")),
    ],
    install_requires=["setuptools", "numpy", "pyyaml"],
    entry_points={"console_scripts": ["dm_mapper = dm.ros_node:main"]},
)

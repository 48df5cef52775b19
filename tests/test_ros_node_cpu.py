"""CPU: ROS-side helpers of the drop-in node (no GPU needed)."""
import math

import numpy as np

from dm.ros_node import Quaternion, yaw_from_quaternion


def reference_euler_to_quaternion(roll, pitch, yaw):
    # formula of server/thymio_project/thymio_project/main.py:31-36
    qx = np.sin(roll / 2) * np.cos(pitch / 2) * np.cos(yaw / 2) - np.cos(roll / 2) * np.sin(pitch / 2) * np.sin(yaw / 2)
    qy = np.cos(roll / 2) * np.sin(pitch / 2) * np.cos(yaw / 2) + np.sin(roll / 2) * np.cos(pitch / 2) * np.sin(yaw / 2)
    qz = np.cos(roll / 2) * np.cos(pitch / 2) * np.sin(yaw / 2) - np.sin(roll / 2) * np.sin(pitch / 2) * np.cos(yaw / 2)
    qw = np.cos(roll / 2) * np.cos(pitch / 2) * np.cos(yaw / 2) + np.sin(roll / 2) * np.sin(pitch / 2) * np.sin(yaw / 2)
    return [qx, qy, qz, qw]


def test_yaw_roundtrip_with_reference_tf_quaternions():
    for yaw in np.linspace(-math.pi + 1e-6, math.pi - 1e-6, 101):
        q = reference_euler_to_quaternion(0.0, 0.0, yaw)
        got = yaw_from_quaternion(Quaternion(*q))
        assert abs(math.remainder(got - yaw, 2 * math.pi)) < 1e-12

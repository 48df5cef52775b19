"""PC-side launch with the GPU mapping stage (drop-in for
server/thymio_project/launch/pc_server.launch.py:12-34).

Same three parts as the reference launch: slam_toolbox (online_async, with
the reference's slam_config.yaml), the thymio_driver node and rviz2.  The
differences:

* slam_toolbox keeps doing what the GPU stage does not replace (scan matching,
  pose graph, loop closure and the map -> odom TF, slam_config.yaml:24,43-69),
  but its grid is published on /slam_toolbox/map instead of /map (a SetRemap
  scoped to its include), so nothing consumes it;
* dm_mapper (dm/ros_node.py, libdm on the GPU) publishes /map from the same
  /scan + TF, with the parameters of the same slam_config.yaml (resolution,
  max_laser_range, map_update_interval and the scan gating) plus the fixed
  grid size, and /frontiers (and /goal_pose with dm_explore:=true);
* ThymioBrain.map_cb (main.py:46,80-81), get_map_image (main.py:241-279) and
  RViz's Map display (rviz_config.rviz:148-165) read /map unchanged.
"""
import os

import yaml
from ament_index_python.packages import get_package_share_directory
from launch import LaunchDescription
from launch.actions import DeclareLaunchArgument, GroupAction, IncludeLaunchDescription
from launch.launch_description_sources import PythonLaunchDescriptionSource
from launch.substitutions import LaunchConfiguration
from launch_ros.actions import Node, SetRemap


def generate_launch_description():
    pkg_thymio = get_package_share_directory('thymio_project')
    slam_config_path = os.path.join(pkg_thymio, 'config', 'slam_config.yaml')
    with open(slam_config_path) as f:
        slam_params = yaml.safe_load(f)['slam_toolbox']['ros__parameters']

    slam_launch = GroupAction([
        SetRemap(src='/map', dst='/slam_toolbox/map'),
        SetRemap(src='/map_metadata', dst='/slam_toolbox/map_metadata'),
        IncludeLaunchDescription(
            PythonLaunchDescriptionSource(
                os.path.join(get_package_share_directory('slam_toolbox'), 'launch', 'online_async_launch.py')
            ),
            launch_arguments={'slam_params_file': slam_config_path}.items()
        ),
    ])

    dm_mapper = Node(
        package='dm_mapping',
        executable='dm_mapper',
        name='dm_mapper',
        output='screen',
        parameters=[slam_params, {
            'dm_width': LaunchConfiguration('dm_width'),
            'dm_height': LaunchConfiguration('dm_height'),
            'dm_device': LaunchConfiguration('dm_device'),
            # e.g. dm_devices:=0,1,2,3,4,5,6,7: one map sharded in row bands
            # over these GPUs (dm_create_sharded); empty: one GPU (dm_device)
            'dm_devices': LaunchConfiguration('dm_devices'),
            'dm_explore': LaunchConfiguration('dm_explore'),
        }],
    )

    thymio_driver = Node(
        package='thymio_project',
        executable='main',
        name='thymio_driver',
        output='screen'
    )

    rviz_node = Node(
        package='rviz2',
        executable='rviz2',
        name='rviz2'
    )

    return LaunchDescription([
        DeclareLaunchArgument('dm_width', default_value='4096'),
        DeclareLaunchArgument('dm_height', default_value='4096'),
        DeclareLaunchArgument('dm_device', default_value='0'),
        DeclareLaunchArgument('dm_devices', default_value=''),
        DeclareLaunchArgument('dm_explore', default_value='false'),
        slam_launch,
        dm_mapper,
        thymio_driver,
        rviz_node,
    ])

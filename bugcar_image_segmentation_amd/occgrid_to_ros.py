"""convert_to_occupancy_grid_msg with the reference's API (occgrid_to_ros.py:13-61).

Host-side message assembly. The flip(0) + rot90-counter-clockwise of the reference
(occgrid_to_ros.py:18-21) is G[::-1, ::-1].T; the GPU rasteriser can emit that order directly
(`bev_transform_tools.create_occupancy_grid_device(..., ros_layout=True)`), in which case pass
`ros_layout=True` here and the array is used as is.

When rospy / nav_msgs are importable the real ROS message types are used; otherwise light
stand-ins with the same field names (so the function runs headless, e.g. in tests and benches).
"""
from __future__ import annotations

import time
from types import SimpleNamespace

import numpy as np
from scipy.spatial.transform import Rotation as R

try:  # pragma: no cover - ROS is not installed in the build image
    import rospy
    from std_msgs.msg import Header
    from nav_msgs.msg import OccupancyGrid, MapMetaData
    from geometry_msgs.msg import Pose, Point, Quaternion
    HAVE_ROS = True
except Exception:  # noqa: BLE001
    rospy = None
    HAVE_ROS = False

    class _Msg(SimpleNamespace):
        pass

    class Header(_Msg):
        def __init__(self):
            super().__init__(seq=0, stamp=None, frame_id="")

    class Point(_Msg):
        def __init__(self):
            super().__init__(x=0.0, y=0.0, z=0.0)

    class Quaternion(_Msg):
        def __init__(self):
            super().__init__(x=0.0, y=0.0, z=0.0, w=1.0)

    class Pose(_Msg):
        def __init__(self):
            super().__init__(position=Point(), orientation=Quaternion())

    class MapMetaData(_Msg):
        def __init__(self):
            super().__init__(map_load_time=None, resolution=0.0, width=0, height=0, origin=Pose())

    class OccupancyGrid(_Msg):
        def __init__(self):
            super().__init__(header=Header(), info=MapMetaData(), data=[])


def _now():
    if HAVE_ROS:
        return rospy.Time.now()
    t = time.time()
    return SimpleNamespace(secs=int(t), nsecs=int((t - int(t)) * 1e9))


def ros_data_order(occ_grid) -> np.ndarray:
    """cv2.flip(g, 0) followed by cv2.rotate(ROTATE_90_COUNTERCLOCKWISE) (occgrid_to_ros.py:18-21)."""
    g = np.asarray(occ_grid)
    return np.ascontiguousarray(g[::-1, ::-1].T)


def convert_to_occupancy_grid_msg(occ_grid, map_resolution, map_width, map_height, time_stamp, frame_id, pose,
                                  ros_layout: bool = False):
    """occgrid_to_ros.py:13-61."""
    map_img = np.asarray(occ_grid) if ros_layout else ros_data_order(occ_grid)
    occupancy_grid = map_img.flatten().tolist()                                 # :24-25

    rot = R.from_euler("xyz", pose[3:])                                         # :27
    r = rot.as_quat()                                                           # :28 (x, y, z, w)
    r_mat = rot.as_matrix()                                                     # :29
    first_cell_in_bev = np.array([0, -map_width / 2, 0]) + pose[:3]             # :30
    first_cell = np.matmul(r_mat, first_cell_in_bev)                            # :31

    msg = OccupancyGrid()
    msg.header = Header()
    msg.header.frame_id = frame_id
    msg.header.stamp = time_stamp
    msg.info = MapMetaData()
    msg.info.height = int(map_width / map_resolution)                          # :39
    msg.info.width = int(map_height / map_resolution)                          # :41
    msg.info.resolution = map_resolution
    msg.info.origin = Pose()
    msg.info.origin.position = Point()
    msg.info.origin.position.x = first_cell[0]
    msg.info.origin.position.y = first_cell[1]
    msg.info.origin.position.z = first_cell[2]
    msg.info.origin.orientation = Quaternion()
    msg.info.origin.orientation.x = r[0]
    msg.info.origin.orientation.y = r[1]
    msg.info.origin.orientation.z = r[2]
    msg.info.origin.orientation.w = r[3]
    msg.data.extend(occupancy_grid)
    msg.info.map_load_time = _now()                                             # :60
    return msg

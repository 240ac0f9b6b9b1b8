"""`import vren` drop-in: put rad-nerf_amd/ on sys.path and the reference's
models/custom_functions.py, rendering.py and ml_rendering.py bind to the HIP
library through this module."""
from radnerf_amd.vren import *  # noqa: F401,F403
from radnerf_amd.vren import (ray_aabb_intersect, raymarching_train, raymarching_test,  # noqa: F401
                              composite_train_fw, composite_train_bw, composite_test_fw,
                              morton3D, morton3D_invert, packbits, distortion_loss_fw,
                              distortion_loss_bw, ray_sphere_intersect)

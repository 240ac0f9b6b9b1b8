"""Ray generation for a training batch (first half):
datasets/ray_utils.py:45-70 (get_rays) and the per-batch pose / pixel gather
of train_ml.py:84-96 as one HIP pass (rn_get_rays)."""
import torch

from ._lib import lib


def _c(t, dtype=torch.float32):
    return t.to(dtype).contiguous()


def get_rays(directions, c2w):
    """ray_utils.get_rays: directions (N,3), c2w (3,4) or (N,3,4) -> rays_o, rays_d."""
    directions = _c(directions)
    n = directions.shape[0]
    dev = directions.device
    rays_o = torch.empty(n, 3, device=dev)
    rays_d = torch.empty(n, 3, device=dev)
    c2w = _c(c2w)
    img = None
    if c2w.ndim == 3:
        img = torch.arange(n, device=dev, dtype=torch.int64)
    lib().get_rays(directions.data_ptr(), c2w.data_ptr(), None if img is None else img.data_ptr(),
                   None, n, None, rays_o.data_ptr(), rays_d.data_ptr(), None,
                   torch.cuda.current_stream(dev).cuda_stream)
    return rays_o, rays_d


def batch_rays(directions, poses, img_idxs, pix_idxs, with_imgs_d=True):
    """train_ml.py:84-96 for split='train': rays_o, rays_d (and imgs_d, the
    pose applied to the mean camera direction) of the picked pixels."""
    directions, poses = _c(directions), _c(poses)
    img_idxs, pix_idxs = _c(img_idxs, torch.int64), _c(pix_idxs, torch.int64)
    n = img_idxs.shape[0]
    dev = directions.device
    rays_o = torch.empty(n, 3, device=dev)
    rays_d = torch.empty(n, 3, device=dev)
    imgs_d = torch.empty(n, 3, device=dev) if with_imgs_d else None
    mean_dir = directions.mean(0).contiguous() if with_imgs_d else None
    lib().get_rays(directions.data_ptr(), poses.data_ptr(), img_idxs.data_ptr(),
                   pix_idxs.data_ptr(), n, None if mean_dir is None else mean_dir.data_ptr(),
                   rays_o.data_ptr(), rays_d.data_ptr(),
                   None if imgs_d is None else imgs_d.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    return (rays_o, rays_d, imgs_d) if with_imgs_d else (rays_o, rays_d)

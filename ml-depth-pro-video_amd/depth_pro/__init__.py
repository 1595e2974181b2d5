"""depth_pro -- MI355X-native Depth Pro inference (drop-in for the reference package).

    import depth_pro
    model, transform = depth_pro.create_model_and_transforms(device=torch.device("cuda:0"))
    image, _, f_px = depth_pro.load_rgb(path)
    prediction = model.infer(transform(image), f_px=f_px)

Same public names as the reference `src/depth_pro/__init__.py:4-5`.
"""

from .depth_pro import (DEFAULT_MONODEPTH_CONFIG_DICT, DepthPro, DepthProConfig,  # noqa: F401
                        create_model_and_transforms)
from .utils import load_rgb  # noqa: F401

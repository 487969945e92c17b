"""Golden SSD anchors from the reference's own generator (BlazePoser/blazeFaceUtils.py, pure Python,
importable in the build container) with the detector's options (blazeFaceDetectorH5.py:232-239).
Writes tests/golden/anchors_blazeface_128.npy [896, 4] = (x_center, y_center, h, w)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main(ref='/root/reference/BlazePoser'):
    sys.path.insert(0, ref)
    from blazeFaceUtils import SsdAnchorsCalculatorOptions, gen_anchors
    o = SsdAnchorsCalculatorOptions(input_size_width=128, input_size_height=128, min_scale=0.1484375,
                                    max_scale=0.75, anchor_offset_x=0.5, anchor_offset_y=0.5, num_layers=4,
                                    feature_map_width=[], feature_map_height=[], strides=[8, 16, 16, 16],
                                    aspect_ratios=[1.0], reduce_boxes_in_lowest_layer=False,
                                    interpolated_scale_aspect_ratio=1.0, fixed_anchor_size=True)
    a = np.asarray([[x.x_center, x.y_center, x.h, x.w] for x in gen_anchors(o)], dtype=np.float64)
    np.save(os.path.join(HERE, 'anchors_blazeface_128.npy'), a)
    print(a.shape)


if __name__ == '__main__':
    main(*sys.argv[1:])

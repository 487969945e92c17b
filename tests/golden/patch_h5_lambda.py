"""Keep one Keras-written SE + MHA + Lambda checkpoint as a fixture: copy
Model-88/Trained-Models-88/ker7z9mv.h5 byte for byte except each Lambda layer's marshalled bytecode,
which is overwritten IN PLACE inside the model_config attribute by the string '<bytecode stripped>'
followed by JSON whitespace up to the same length.  Every other byte (the HDF5 structure libhdf5
wrote, the weights, the optimizer state) is the file Keras 2.13 wrote; tests/test_h5io.py reads it.

    python tests/golden/patch_h5_lambda.py [/root/reference/Model-88/Trained-Models-88/ker7z9mv.h5]
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = '/root/reference/Model-88/Trained-Models-88/ker7z9mv.h5'
OUT = os.path.join(HERE, 'h5_keras', 'ker7z9mv.h5')
PLACEHOLDER = b'"<bytecode stripped>"'


def patch(raw):
    out = bytearray(raw)
    n = 0
    for m in re.finditer(rb'"function": \["', raw):
        a = m.end() - 1                      # the opening quote of the base64 string
        b = raw.index(b'"', a + 1) + 1       # past its closing quote (base64 + \n escapes, no quotes)
        if b - a < len(PLACEHOLDER):
            raise ValueError('bytecode string shorter than the placeholder')
        out[a:b] = PLACEHOLDER + b' ' * (b - a - len(PLACEHOLDER))
        n += 1
    return bytes(out), n


if __name__ == '__main__':
    src = sys.argv[1] if len(sys.argv) > 1 else SRC
    raw = open(src, 'rb').read()
    out, n = patch(raw)
    assert len(out) == len(raw) and n >= 1
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, 'wb') as f:
        f.write(out)
    print('%s: %d Lambda functions overwritten in place, %d bytes' % (OUT, n, len(out)))

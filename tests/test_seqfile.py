"""Siril .seq files (sg_seqfile_*, src/io/seqfile.c:43-357): the reference's line formats
read and written, old-format I / R lines, the %g precision of cached statistics, and the
selection count fix-up.  Host-only (no GPU)."""
import numpy as np
import pytest

import sirilgpu as sg

SAMPLE = """#Siril sequence file. Contains list of files (images), selection, and registration data
#S 'sequence_name' start_index nb_images nb_selected fixed_len reference_image
S 'pp_light_' 1 4 9 5 2
L 1
I 1 1 1012.37 1001 33.5 21.2 20 31.1 1000.42 29.9511 0 65535
I 2 0
I 3 1 1013.1 1002 33.1 21.4 20 31.4 1001.17 30.0125 0 65535
I 4 1 1011.9 1000 33.9 21.1 20 30.9 999.875 29.8733 0 65535
R0 0 0 0 0 0 0 0.845
R0 -3 5 0 0 0 0 1
R0 2 -7 0 0 0 0 0.5
R0 11 1 0.25
"""


def test_read_reference_format(tmp_path):
    p = tmp_path / "pp_light_.seq"
    p.write_text(SAMPLE)
    with sg.SeqFile.read(str(tmp_path / "pp_light_")) as sf:    # name without .seq (:55-60)
        info = sf.info()
        assert info.name == b"pp_light_" and (info.beg, info.number, info.fixed, info.reference_image) == (1, 4, 5, 2)
        assert info.selnum == 3              # fixed to the actual selection (:253-259)
        assert info.nb_layers == 1 and info.type == sg.SEQFILE_REGULAR
        fn, inc, hs, st = sf.images()
        assert fn.tolist() == [1, 2, 3, 4] and inc.tolist() == [1, 0, 1, 1] and hs.tolist() == [1, 0, 1, 1]
        assert st[0, 6] == 1000.42 and st[0, 7] == 29.9511 and st[3, 6] == 999.875
        rc, sx, sy, rcx, rcy, ang, fw, q = sf.registration(0)
        assert rc == 0
        assert sx.tolist() == [0, -3, 2, 11] and sy.tolist() == [0, 5, -7, 1]
        assert q.tolist() == [0.845, 1.0, 0.5, 0.0]    # old 3-token line: third token dropped (:158-163)
        assert rcx[3] == 0.0


def test_write_read_round_trip(tmp_path):
    with sg.SeqFile.create("r_seq", 3, beg=0, reference_image=1, type=sg.SEQFILE_SER, nb_layers=3) as sf:
        sf.set_image(1, 1, 0)
        sf.set_image(2, 2, 1, stats=[1.5, 2, 3, 4, 5, 6, 1000.123456789, 29.987654321, 0, 65535])
        sf.set_registration(1, [0, 4, -2], [0, -1, 9], quality=[1.0, 0.25, 0.5])
        path = str(tmp_path / "r_seq.seq")
        sf.write(path)
    text = open(path).read().splitlines()
    assert text[2] == "S 'r_seq' 0 3 2 5 1" and text[3] == "TS" and text[4] == "L 3"
    assert text[5] == "I 0 1" and text[6] == "I 1 0"
    assert text[7] == "I 2 1 1.5 2 3 4 5 6 1000.12 29.9877 0 65535"     # %g: six significant digits
    assert text[8:] == ["R1 0 0 0 0 0 0 1", "R1 4 -1 0 0 0 0 0.25", "R1 -2 9 0 0 0 0 0.5"]
    with sg.SeqFile.read(path) as sf:
        info = sf.info()
        assert info.type == sg.SEQFILE_SER and info.nb_layers == 3 and info.selnum == 2
        assert sf.registration(0)[0] == 1 and sf.registration(2)[0] == 1
        rc, sx, sy, *_, q = sf.registration(1)
        assert rc == 0 and sx.tolist() == [0, 4, -2] and sy.tolist() == [0, -1, 9] and q.tolist() == [1.0, 0.25, 0.5]
        st = sf.images()[3]
        assert st[2, 6] == 1000.12 and st[2, 7] == 29.9877


@pytest.mark.parametrize("bad", ["S 'x' 1 0 0 5 -1\nL 1\n", "L 1\nI 1 1\n", "S 'x' 1 1 1 5 -1\nL 1\nI 1 1 2 3\n",
                                 "S 'x' 1 1 1 5 -1\nL 1\nR3 0 0 0 0 0 0 1\n",
                                 "S 'x' 1 -5 0 5 -1\nL 1\n",            # negative image count
                                 "S 'x' 1 2 0 5 -1\nL -1\n",            # negative layer count
                                 "S 'x' 1 2000000000 0 5 -1\nL 1\n"])   # allocation too large
def test_malformed(tmp_path, bad):
    p = tmp_path / "bad.seq"
    p.write_text(bad)
    with pytest.raises(OSError):
        sg.SeqFile.read(str(p))

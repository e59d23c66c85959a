"""Data of the synchronised cell-population cases (tests/test_cellpop_sync*.py): the time-course
fixture (cellpop_tc_data.json) plus two courses on time axes relative to a synchronisation point,
as DataLikelihoodTimeCourse / DataLikelihoodTimePoints read them with synchronize="..."
(src/cellpop/DataLikelihoodTimeCourse.cpp:27-41, 190-199):
  tsync = -6 .. 4 h (every 2 h), pcna_sync[tsync][cell]: 16 observed cells (rows 8..13 of pcna_cells)
  tneg  = -6 .. -1 h (every 1 h), pcna_neg[tneg][cell]:  16 observed cells (rows 4..9 of pcna_cells)
Both have time points before the synchronisation point, so the experiment also simulates their
full duration (the entry of .cpp:192-199). The values are observations for parity tests only.

Also cellpop_lineage_data.json: the time-course fixture plus an observed lineage over its 16
pcna_cells (DataLikelihoodTimeCourse.cpp:132-167): "cell_id" 100..115 and "parent" (INT_MIN = none):
cells 0..7 are roots; 8 and 9 are children of cell 0, 10 of 1, 11 of 2, 12 of 3, 13 of 8 (a
grandchild), 14 of 4, 15 of 5.

    python tests/golden/make_cellpop_sync_data.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    with open(os.path.join(HERE, "cellpop_tc_data.json")) as f:
        d = json.load(f)
    g = d["exp1"]
    cells = g["pcna_cells"]["data"]  # [21 time points][16 cells]
    g["tsync"] = {"dims": ["tsync"], "data": [-6.0, -4.0, -2.0, 0.0, 2.0, 4.0]}
    g["pcna_sync"] = {"dims": ["tsync", "cell"], "data": cells[8:14]}
    g["tneg"] = {"dims": ["tneg"], "data": [-6.0, -5.0, -4.0, -3.0, -2.0, -1.0]}
    g["pcna_neg"] = {"dims": ["tneg", "cell"], "data": cells[4:10]}
    with open(os.path.join(HERE, "cellpop_sync_data.json"), "w") as f:
        json.dump(d, f)
    with open(os.path.join(HERE, "cellpop_tc_data.json")) as f:
        lin = json.load(f)
    INT_MIN = -2147483648
    parent_of = {8: 0, 9: 0, 10: 1, 11: 2, 12: 3, 13: 8, 14: 4, 15: 5}
    lin["exp1"]["cell_id"] = {"dims": ["cell"], "data": [100 + i for i in range(16)]}
    lin["exp1"]["parent"] = {"dims": ["cell"], "data": [100 + parent_of[i] if i in parent_of else INT_MIN for i in range(16)]}
    with open(os.path.join(HERE, "cellpop_lineage_data.json"), "w") as f:
        json.dump(lin, f)


if __name__ == "__main__":
    main()

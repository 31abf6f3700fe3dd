"""CPU: the MovieLens feature builder (createRatingDataFrame, FactorizationMachinesSample.scala:
75-128) on a hand-checked example (the dataset itself is not available offline)."""

import numpy as np

from fm_spark_amd.data import MAX_MOVIE_ID, MAX_USER_ID, movielens_features, read_ratings_csv


def test_hand_example(tmp_path):
    p = tmp_path / "ratings.csv"
    # user 1 rates movies 10, 20, 30; user 2 rates movie 10 only; user 1 rates 20 twice (same rating)
    p.write_text("userId,movieId,rating,timestamp\n1,10,4.0,1\n1,20,3.5,2\n1,30,5.0,3\n2,10,2.0,4\n1,20,3.5,9\n")
    u, m, r = read_ratings_csv(str(p))
    labels, row_ptr, col, val, size = movielens_features(u, m, r)
    assert size == MAX_USER_ID + 2 * MAX_MOVIE_ID
    np.testing.assert_array_equal(labels, [4.0, 3.5, 5.0, 2.0])
    rows = [dict(zip(col[a:b].tolist(), val[a:b].tolist())) for a, b in zip(row_ptr[:-1], row_ptr[1:])]
    base = MAX_USER_ID + MAX_MOVIE_ID
    assert rows[0] == {1: 1.0, MAX_USER_ID + 10: 1.0, base + 20: 0.5, base + 30: 0.5}
    assert rows[1] == {1: 1.0, MAX_USER_ID + 20: 1.0, base + 10: 0.5, base + 30: 0.5}
    assert rows[2] == {1: 1.0, MAX_USER_ID + 30: 1.0, base + 10: 0.5, base + 20: 0.5}
    assert rows[3] == {2: 1.0, MAX_USER_ID + 10: 1.0}  # a set of one: no implicit-feedback part
    for a, b in zip(row_ptr[:-1], row_ptr[1:]):
        assert np.all(np.diff(col[a:b]) > 0)


def test_same_movie_two_ratings():
    # two distinct "movieId:rating" strings of one movie: both rows, each sees the other's movie
    # id == its own, which the filter drops, so only the third movie remains (weight 1/2)
    labels, row_ptr, col, val, _ = movielens_features([5, 5, 5], [7, 7, 8], [1.0, 2.0, 3.0])
    rows = [dict(zip(col[a:b].tolist(), val[a:b].tolist())) for a, b in zip(row_ptr[:-1], row_ptr[1:])]
    base = MAX_USER_ID + MAX_MOVIE_ID
    assert labels.tolist() == [1.0, 2.0, 3.0]
    assert rows[0] == {5: 1.0, MAX_USER_ID + 7: 1.0, base + 8: 0.5}
    assert rows[2] == {5: 1.0, MAX_USER_ID + 8: 1.0, base + 7: 0.5}

"""DB sources/sinks on the embedded SQLite engine (reference DerbyDB / JdbcDB role), the JDBC retract
(upsert) sink, and WindowGroupByStreamOp (TUMBLE / HOP / SESSION over an event-time column)."""
import os

from alink_amd import *  # noqa: F401,F403


def test_db_batch_and_stream_round_trip(tmp_path):
    db = SqliteDB(os.path.join(str(tmp_path), "t.db"))
    src = MemSourceBatchOp([(1, "a", 1.5), (2, "b", 2.5)], "id bigint, name string, v double")
    src.link(DBSinkBatchOp(db, "tbl"))
    assert db.listTableNames() == ["tbl"]
    assert [tuple(r) for r in DBSourceBatchOp(db, "tbl").collect()] == [(1, "a", 1.5), (2, "b", 2.5)]
    MemSourceStreamOp([(1, "x", 9.0), (3, "c", 3.5)], "id bigint, name string, v double") \
        .link(JdbcRetractSinkStreamOp(db, "up", ["id"]))
    StreamOperator.execute()
    MemSourceStreamOp([(1, "y", 10.0)], "id bigint, name string, v double") \
        .link(JdbcRetractSinkStreamOp(db, "up", ["id"]))
    StreamOperator.execute()
    assert sorted(tuple(r) for r in DBSourceBatchOp(db, "up").collect()) == [(1, "y", 10.0), (3, "c", 3.5)]
    box = []
    DBSourceStreamOp(db, "tbl").link(CollectStreamOp(box))
    StreamOperator.execute()
    assert [tuple(r) for r in box] == [(1, "a", 1.5), (2, "b", 2.5)]


ROWS = [(0.5, "a", 1.0), (1.2, "a", 2.0), (1.7, "b", 3.0), (2.1, "a", 4.0), (4.0, "b", 5.0)]


def _run(op):
    box = []
    op.linkFrom(MemSourceStreamOp(ROWS, "ts double, k string, v double")).link(CollectStreamOp(box))
    StreamOperator.execute()
    return [tuple(r) for r in box]


def test_window_group_by():
    """Aggregates per window plus the reference's window_start / window_end TIMESTAMP columns
    (WindowGroupByStreamOp.java:80-82; WindowGroupByStreamOpTest: 2 selected + 2 window columns)."""
    def split(rows):
        return [r[:-2] for r in rows], [(r[-2].timestamp(), r[-1].timestamp()) for r in rows]
    tumble, win = split(_run(WindowGroupByStreamOp().setTimeCol("ts").setWindowLength(1)
                             .setSelectClause("k, SUM(v) AS s, COUNT(*) AS c").setGroupByClause("k")))
    assert tumble == [("a", 1.0, 1), ("a", 2.0, 1), ("b", 3.0, 1), ("a", 4.0, 1), ("b", 5.0, 1)]
    assert win == [(0.0, 1.0), (1.0, 2.0), (1.0, 2.0), (2.0, 3.0), (4.0, 5.0)]
    session, win = split(_run(WindowGroupByStreamOp().setTimeCol("ts").setWindowType("SESSION").setSessionGap(1)
                              .setSelectClause("SUM(v) AS s")))
    assert session == [(10.0,), (5.0,)]
    assert win == [(0.5, 3.1), (4.0, 5.0)]                   # session end = last event + gap
    hop, win = split(_run(WindowGroupByStreamOp().setTimeCol("ts").setWindowType("HOP").setWindowLength(2)
                          .setSlidingLength(1).setSelectClause("SUM(v) AS s")))
    assert hop == [(1.0,), (6.0,), (9.0,), (4.0,), (5.0,), (5.0,)]
    assert all(e - s == 2.0 for s, e in win)


def test_kafka_file_broker_and_hive_local_warehouse(tmp_path):
    broker = "file://" + str(tmp_path / "kafka")
    MemSourceStreamOp([(1, "a", 1.5), (2, "b", 2.5)], "id bigint, name string, v double") \
        .link(KafkaSinkStreamOp().setBootstrapServers(broker).setTopic("t1"))
    StreamOperator.execute()
    box = []
    KafkaSourceStreamOp().setBootstrapServers(broker).setTopic("t1").setStartupMode("EARLIEST") \
        .link(CollectStreamOp(box))
    StreamOperator.execute()
    assert [tuple(r) for r in box] == [(None, '{"id":1,"name":"a","v":1.5}', "t1", 0, 0),
                                       (None, '{"id":2,"name":"b","v":2.5}', "t1", 0, 1)]
    wh = "file://" + str(tmp_path / "hive")
    MemSourceBatchOp([(1, "a")], "id bigint, s string").link(
        HiveSinkBatchOp().setHiveConfDir(wh).setOutputTableName("ht").setPartition("ds=1"))
    MemSourceBatchOp([(2, "b")], "id bigint, s string").link(
        HiveSinkBatchOp().setHiveConfDir(wh).setOutputTableName("ht").setPartition("ds=2"))
    assert [tuple(r) for r in HiveSourceBatchOp().setHiveConfDir(wh).setInputTableName("ht")
            .setPartitions("ds=2").collect()] == [(2, "b")]
    assert len(HiveSourceBatchOp().setHiveConfDir(wh).setInputTableName("ht").collect()) == 2

/*
 * skc.gpu.NativeKmerCounter -- Scala side of jni/fastkmer_jni.c.
 *
 * The drop-in for the body of SparkBinKmerCounter.executeJob
 * (src/main/scala/skc/SparkBinKmerCounter.scala:989-1046): one MI355X context per
 * executor runs the map (getSuperKmers, :34-169), the bin shuffle (reduceByKey,
 * :1034-1042) and the per-bin count (extractKXmers / extractKXmersHT, :428-660,
 * :664-739) and writes the same bin<b> files.  TestConfiguration is the reference's
 * skc.test.testutil.TestConfiguration (src/main/scala/skc/test/package.scala:16-42).
 * Not compiled in this repository (no JVM in the image); see INTEGRATION.md.
 */
package skc.gpu

import skc.test.testutil.TestConfiguration

object NativeKmerCounter {
  System.loadLibrary("fastkmer_jni") // libfastkmer_jni.so, linked against libfastkmer.so

  @native def create(k: Int, m: Int, x: Int, b: Int, useHT: Boolean, sequenceType: Int,
                     nRanks: Int, rank: Int, device: Int): Long
  @native def ingest(h: Long, fasta: java.nio.ByteBuffer, n: Long, last: Boolean): Unit
  @native def ingestFileRange(h: Long, path: String, world: Int, rank: Int, window: Long): Unit
  @native def balanceBinsFile(h: Long, path: String, world: Int, rank: Int, fraction: Double): Unit
  @native def finish(h: Long): Unit
  @native def commUniqueId(): Array[Byte]
  @native def commInit(h: Long, id: Array[Byte]): Unit
  @native def binSizes(h: Long): Array[Long]
  @native def writeBins(h: Long, outDir: String): Unit
  @native def findBinSignatures(h: Long, outDir: String): Unit
  @native def destroy(h: Long): Unit

  /** The whole file as the job's input, read by the library (fk_ingest_file_range: positioned
    * reads into pinned windows, each copied and mapped while the next is read). */
  private def ingestFile(h: Long, dataset: String, window: Long): Unit =
    ingestFileRange(h, dataset, 1, 0, window)

  def executeJob(configuration: TestConfiguration, device: Int = -1, window: Long = 1L << 28): Unit = {
    val h = create(configuration.k, configuration.m, configuration.x, configuration.b,
      configuration.useHT, configuration.sequenceType, 1, 0, device)
    try {
      ingestFile(h, configuration.dataset, window)
      finish(h)
      if (configuration.write) writeBins(h, configuration.outputDir)
    } finally destroy(h)
  }

  /** One rank of an nRanks-GPU job (one executor per GPU): `commId` comes from commUniqueId()
    * on one node and reaches every rank with the task (a broadcast variable).  The rank reads its
    * own split of `configuration.dataset` -- the library cuts it as FASTdoop's input formats do
    * (SBKC:993, 1009-1012): whole records for sequenceType 0; for sequenceType 1 the rank's byte
    * range with a header prefix and the k - 1 overlap -- and streams it in windows of `window`
    * bytes (any split size: no 2 GiB mapping limit).  The records move between the GPUs inside
    * ingest / finish (RCCL all-to-all over xGMI, the reduceByKey of :1034-1042); each rank writes
    * the bin files of the bins it owns into the shared output directory: bin % nRanks == rank, or
    * with configuration.useCustomPartitioner the LPT placement of the reference's partitioner
    * (SBKC:1023-1026; MultiprocessorSchedulingPartitioner.scala:35-69) computed from a 1 % sample
    * of every rank's split (sample(false, 0.01), SBKC:1024) before the job's input is read. */
  def executeJobRank(configuration: TestConfiguration, rank: Int, nRanks: Int, commId: Array[Byte],
                     device: Int = -1, window: Long = 1L << 28): Array[Long] = {
    val h = create(configuration.k, configuration.m, configuration.x, configuration.b,
      configuration.useHT, configuration.sequenceType, nRanks, rank, device)
    try {
      commInit(h, commId)
      if (configuration.useCustomPartitioner)
        balanceBinsFile(h, configuration.dataset, nRanks, rank, 0.01)
      ingestFileRange(h, configuration.dataset, nRanks, rank, window)
      finish(h)
      if (configuration.write) writeBins(h, configuration.outputDir)
      binSizes(h)
    } finally destroy(h)
  }

  /** SparkBinKmerCounter.executeFindBinSignaturesJob (:956-986): bin_signatures<b>.txt. */
  def executeFindBinSignaturesJob(configuration: TestConfiguration, device: Int = -1,
                                  window: Long = 1L << 28): Unit = {
    val h = create(configuration.k, configuration.m, configuration.x, configuration.b,
      configuration.useHT, configuration.sequenceType, 1, 0, device)
    try {
      ingestFile(h, configuration.dataset, window)
      findBinSignatures(h, configuration.outputDir)
    } finally destroy(h)
  }
}

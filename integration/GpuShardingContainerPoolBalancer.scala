/*
 * Drop-in LoadBalancerProvider for the MI355X engine (SOURCE ONLY: this image has no JDK/scalac, see DESIGN.md).
 *
 * A maintainer adds this file to core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/ and selects
 * it with   whisk.spi.LoadBalancerProvider = org.apache.openwhisk.core.loadBalancer.GpuShardingContainerPoolBalancer
 * (common/scala/src/main/resources/reference.conf:26, or CONFIG_whisk_spi_LoadBalancerProvider).
 *
 * Everything except the scheduling state stays as in ShardingContainerPoolBalancer (SCPB): CommonLoadBalancer keeps
 * activation bookkeeping, the Kafka send, the ack feed and processCompletion; the monitor actor keeps forwarding
 * CurrentInvokerPoolState and cluster membership (including cluster bootstrap, SCPB:159-167); the capacity/health gauges
 * (SCPB:169-205) and the per-activation logs (SCPB:299-301, 312-314) are emitted as the reference does.  publish()
 * enqueues into a single batching thread that owns the native context (single writer, owgs.h "Threading");
 * releaseInvoker() enqueues into the same thread.  Each drained batch goes to the engine as ONE owgs_process_batch
 * call (runs of completions then publishes, in queue order) through direct ByteBuffers: no JVM array is pinned across
 * the GPU round trip.
 */
package org.apache.openwhisk.core.loadBalancer

import java.nio.{ByteBuffer, ByteOrder}
import java.util.concurrent.{ArrayBlockingQueue, TimeUnit}

import akka.actor.{Actor, ActorRef, ActorRefFactory, ActorSystem, Props}
import akka.cluster.ClusterEvent._
import akka.cluster.{Cluster, Member, MemberStatus}
import akka.management.scaladsl.AkkaManagement
import akka.management.cluster.bootstrap.ClusterBootstrap
import akka.stream.ActorMaterializer
import org.apache.kafka.clients.producer.RecordMetadata
import pureconfig._
import pureconfig.generic.auto._
import org.apache.openwhisk.common._
import org.apache.openwhisk.common.LoggingMarkers._
import org.apache.openwhisk.core.WhiskConfig._
import org.apache.openwhisk.core.connector._
import org.apache.openwhisk.core.entity._
import org.apache.openwhisk.core.entity.size.SizeLong
import org.apache.openwhisk.core.loadBalancer.InvokerState.{Healthy, Offline, Unhealthy, Unresponsive}
import org.apache.openwhisk.core.{ConfigKeys, WhiskConfig}
import org.apache.openwhisk.spi.SpiLoader

import scala.collection.mutable
import scala.concurrent.{Future, Promise}

/** JNI surface of libowgs.so (include/owgs.h); implemented by integration/owgs_jni.c. */
object OwgsNative {
  System.loadLibrary("owgs_jni")
  @native def create(managedFraction: Double, blackboxFraction: Double, minMemoryBytes: Long, clusterSize: Int,
                     device: Int, rngSeed: Long): Long
  @native def destroy(ctx: Long): Unit
  @native def updateInvokers(ctx: Long, ids: Array[Int], userMemoryBytes: Array[Long], status: Array[Byte]): Int
  @native def updateCluster(ctx: Long, size: Int): Int
  @native def registerAction(ctx: Long, namespace: String, path: String, key: String, memMb: Int, maxConc: Int,
                             blackbox: Boolean): Int
  /** owgs_process_batch over direct buffers (native byte order), layout in BatchBuffers; the publishes' overload-RNG
   *  sequence numbers are seqBase, seqBase + 1, ... in queue order. */
  @native def processBatch(ctx: Long, in: ByteBuffer, out: ByteBuffer, nRuns: Int, nRel: Int, nPub: Int,
                           seqBase: Long): Int
  /** owgs_release_actions: handles of cold fqn@version keys (none of their activations in flight) */
  @native def releaseActions(ctx: Long, handles: Array[Int], n: Int): Int
  @native def lastError(ctx: Long): String
}

/** The direct buffers of one drained batch (owgs_jni.c processBatch reads the same layout):
 *  in  = relOff[nRuns + 1], pubOff[nRuns + 1], relInvoker[nRel], relAction[nRel], pubAction[nPub] (ints);
 *  out = outInvoker[nPub] (ints), outFlags[nPub], relFlags[nRel] (bytes). */
final class BatchBuffers {
  var in: ByteBuffer = ByteBuffer.allocateDirect(1 << 16).order(ByteOrder.nativeOrder())
  var out: ByteBuffer = ByteBuffer.allocateDirect(1 << 15).order(ByteOrder.nativeOrder())
  def ensure(nRuns: Int, nRel: Int, nPub: Int): Unit = {
    val inBytes = 4L * (2 * (nRuns + 1) + 2 * nRel + nPub)
    val outBytes = 4L * nPub + nPub + nRel
    if (inBytes > in.capacity) in = ByteBuffer.allocateDirect((2 * inBytes).toInt).order(ByteOrder.nativeOrder())
    if (outBytes > out.capacity) out = ByteBuffer.allocateDirect((2 * outBytes).toInt).order(ByteOrder.nativeOrder())
    in.clear()
    out.clear()
  }
}

class GpuShardingContainerPoolBalancer(config: WhiskConfig,
                                       controllerInstance: ControllerInstanceId,
                                       feedFactory: FeedFactory,
                                       val invokerPoolFactory: InvokerPoolFactory,
                                       implicit val messagingProvider: MessagingProvider =
                                         SpiLoader.get[MessagingProvider])(implicit actorSystem: ActorSystem,
                                                                           logging: Logging,
                                                                           materializer: ActorMaterializer)
    extends CommonLoadBalancer(config, feedFactory, controllerInstance) {

  /** Build a cluster of all loadbalancers, exactly as SCPB:159-167 does (bootstrap, seed nodes, or none). */
  private val cluster: Option[Cluster] = if (loadConfigOrThrow[ClusterConfig](ConfigKeys.cluster).useClusterBootstrap) {
    AkkaManagement(actorSystem).start()
    ClusterBootstrap(actorSystem).start()
    Some(Cluster(actorSystem))
  } else if (loadConfigOrThrow[Seq[String]]("akka.cluster.seed-nodes").nonEmpty) {
    Some(Cluster(actorSystem))
  } else {
    None
  }

  // device and overload-RNG seed of this controller: whisk.loadbalancer.gpu.{device, rng-seed} (optional keys)
  private val gpuConfig = actorSystem.settings.config
  private def cfgInt(k: String, d: Int): Int = if (gpuConfig.hasPath(k)) gpuConfig.getInt(k) else d
  private def cfgLong(k: String, d: Long): Long = if (gpuConfig.hasPath(k)) gpuConfig.getLong(k) else d
  private val ctx = OwgsNative.create(lbConfig.managedFraction, lbConfig.blackboxFraction,
    MemoryLimit.MIN_MEMORY.toBytes, 1, cfgInt("whisk.loadbalancer.gpu.device", 0),
    cfgLong("whisk.loadbalancer.gpu.rng-seed", controllerInstance.asString.hashCode.toLong))
  require(ctx != 0L, "owgs_create failed (no MI355X visible or libowgs.so missing)")

  // SCPB:467-468: the fractions the state uses (also for the pool views below)
  private val managedFraction: Double = Math.max(0.0, Math.min(1.0, lbConfig.managedFraction))
  private val blackboxFraction: Double = Math.max(1.0 - managedFraction, Math.min(1.0, lbConfig.blackboxFraction))

  // (invoking namespace, fqn@version) -> native action handle (registered once); fqn@version -> a handle of that
  // action for releases (a release only needs the NestedSemaphore key and the limits, NS:98-113).  Per key: the
  // handles naming it, its activations in flight and the last batch that used it; keys idle for keyIdleBatches with
  // nothing in flight give their handles back (owgs_release_actions), as the reference's NestedSemaphore drops the
  // key's entries at operationCount 0 (NestedSemaphore.scala:109-111): every action update bumps the version, so the
  // set of keys a controller sees over its lifetime is unbounded.
  private val handles = mutable.HashMap.empty[(String, String), Int]
  private val byKey = mutable.HashMap.empty[String, Int]
  private final class KeyUse(var inFlight: Int, var lastBatch: Long, val names: mutable.ArrayBuffer[(String, String)])
  private val keyUse = mutable.HashMap.empty[String, KeyUse]
  private var batchNo = 0L
  private val keyIdleBatches = cfgInt("whisk.loadbalancer.gpu.key-idle-batches", 100000).toLong

  /** The invoker list the engine schedules against, its pools (SCPB:518-523) and userMemory by id, published by the
   *  batching thread right after owgs_update_invokers succeeded (so a decision and the InvokerInstanceId it returns
   *  come from the same list, as schedule() takes both from `invokers(index)`, SCPB:411-414). */
  private final case class Pools(all: IndexedSeq[InvokerHealth], managed: IndexedSeq[InvokerHealth],
                                 blackbox: IndexedSeq[InvokerHealth], byId: Array[InvokerInstanceId])
  @volatile private var pools = Pools(IndexedSeq.empty, IndexedSeq.empty, IndexedSeq.empty, Array.empty)
  @volatile private var _clusterSize = 1

  private def poolsOf(s: IndexedSeq[InvokerHealth]): Pools = {
    val managed = Math.max(1, Math.ceil(s.size.toDouble * managedFraction).toInt)
    val blackboxes = Math.max(1, Math.floor(s.size.toDouble * blackboxFraction).toInt)
    // the pool's own InvokerInstanceId by id: schedule() returns invokers(index).id (SCPB:411-414), uniqueName and
    // displayedName included (InstanceId.scala:31-37)
    val byId = new Array[InvokerInstanceId](if (s.isEmpty) 0 else s.map(_.id.toInt).max + 1)
    s.foreach(h => byId(h.id.toInt) = h.id)
    Pools(s, s.take(managed), s.takeRight(blackboxes), byId)
  }

  private sealed trait Job
  private case class Pub(action: ExecutableWhiskActionMetaData, msg: ActivationMessage,
                         p: Promise[Option[(InvokerInstanceId, Boolean)]]) extends Job
  private case class Rel(invoker: InvokerInstanceId, entry: ActivationEntry) extends Job
  private case class Inv(state: IndexedSeq[InvokerHealth]) extends Job
  private case class Clu(size: Int) extends Job

  private val queue = new ArrayBlockingQueue[Job](1 << 16)
  private var seqNo = 0L  // overload-RNG sequence numbers, given in queue order by the batching thread
  private val bufs = new BatchBuffers

  private def nativeError(what: String, rc: Int): LoadBalancerException =
    LoadBalancerException(s"$what failed ($rc): ${OwgsNative.lastError(ctx)}")

  /** One drained batch of jobs, in queue order (the sequential order the engine replays).  State updates are applied
   *  between segments; each segment of (completions, publishes) runs is ONE owgs_process_batch call. */
  private def runBatch(jobs: java.util.ArrayList[Job]): Unit = {
    val segment = mutable.ArrayBuffer.empty[(mutable.ArrayBuffer[Rel], mutable.ArrayBuffer[Pub])]
    def flush(): Unit = if (segment.nonEmpty) { processSegment(segment); segment.clear() }
    var i = 0
    while (i < jobs.size) {
      jobs.get(i) match {
        case Inv(s) =>
          flush()
          val rc = OwgsNative.updateInvokers(ctx, s.map(_.id.toInt).toArray, s.map(_.id.userMemory.toBytes).toArray,
            s.map(h => statusCode(h.status)).toArray)
          if (rc < 0) logging.error(this, s"updateInvokers: ${nativeError("owgs_update_invokers", rc).getMessage}")
          else pools = poolsOf(s)
          i += 1
        case Clu(n) =>
          flush()
          val rc = OwgsNative.updateCluster(ctx, n)
          if (rc < 0) logging.error(this, s"updateCluster: ${nativeError("owgs_update_cluster", rc).getMessage}")
          else _clusterSize = math.max(1, n)
          i += 1
        case _ =>
          // maximal run of releases followed by publishes, order preserved
          val rels = mutable.ArrayBuffer.empty[Rel]
          while (i < jobs.size && jobs.get(i).isInstanceOf[Rel]) { rels += jobs.get(i).asInstanceOf[Rel]; i += 1 }
          val pubs = mutable.ArrayBuffer.empty[Pub]
          while (i < jobs.size && jobs.get(i).isInstanceOf[Pub]) { pubs += jobs.get(i).asInstanceOf[Pub]; i += 1 }
          segment += ((rels, pubs))
      }
    }
    flush()
  }

  /** releaseInvoker (SCPB:327-331) and the schedule() half of publish (SCPB:260-290) for the runs of one segment, in
   *  one native call.  What the reference would throw from NestedSemaphore.releaseConcurrent / ForcibleSemaphore
   *  .release is logged per release (processCompletion's future fails there too). */
  private def processSegment(runs: mutable.ArrayBuffer[(mutable.ArrayBuffer[Rel], mutable.ArrayBuffer[Pub])]): Unit = {
    // handles first: a publish whose action cannot be registered fails alone
    val planned = runs.map { case (rels, pubs) =>
      val known = rels.filter(r => byKey.contains(r.entry.fullyQualifiedEntityName.asString))
      val ok = pubs.flatMap { p =>
        val h = handleOf(p.msg.user.namespace.name.asString, p.action.fullyQualifiedName(true),
          p.action.limits.memory.megabytes, p.action.limits.concurrency.maxConcurrent, p.action.exec.pull)
        if (h < 0) { p.p.failure(nativeError("owgs_register_actions", h)); None } else Some((p, h))
      }
      (known, ok)
    }
    val nRuns = planned.length
    val nRel = planned.map(_._1.length).sum
    val nPub = planned.map(_._2.length).sum
    if (nRel + nPub == 0) return
    bufs.ensure(nRuns, nRel, nPub)
    val in = bufs.in.asIntBuffer()
    var acc = 0
    in.put(0); planned.foreach { case (r, _) => acc += r.length; in.put(acc) }
    acc = 0
    in.put(0); planned.foreach { case (_, p) => acc += p.length; in.put(acc) }
    planned.foreach(_._1.foreach(r => in.put(r.invoker.toInt)))
    planned.foreach(_._1.foreach(r => in.put(byKey(r.entry.fullyQualifiedEntityName.asString))))
    planned.foreach(_._2.foreach { case (_, h) => in.put(h) })
    // overload-RNG sequence numbers in queue order (the engine's counter RNG replaces ThreadLocalRandom, SCPB:421)
    val seqBase = seqNo
    seqNo += nPub
    val rc = OwgsNative.processBatch(ctx, bufs.in, bufs.out, nRuns, nRel, nPub, seqBase)
    val pubsInOrder = planned.flatMap(_._2.map(_._1))
    if (rc < 0) {
      val e = nativeError("owgs_process_batch", rc)
      logging.error(this, s"process batch: ${e.getMessage}")
      pubsInOrder.foreach(_.p.failure(e))
      return
    }
    val out = bufs.out
    val byId = pools.byId
    var k = 0
    while (k < nPub) {
      val p = pubsInOrder(k)
      val id = out.getInt(4 * k)
      val overload = (out.get(4 * nPub + k) & 1) != 0
      if (id >= 0) {
        val invoker = if (id < byId.length && byId(id) != null) byId(id) else InvokerInstanceId(id, userMemory = 0.B)
        if (overload) // SCPB:423 (logged where schedule() forces the random healthy invoker)
          logging.warn(this, s"system is overloaded. Chose invoker${id} by random assignment.")(p.msg.transid)
        keyUse.get(p.action.fullyQualifiedName(true).asString).foreach(_.inFlight += 1)
        p.p.success(Some((invoker, overload)))
      } else if (id == -2) // the reference's schedule() throws here (Int.MinValue hash or an id outside invokerSlots)
        p.p.failure(new IndexOutOfBoundsException(s"schedule: invoker index out of range for activation ${p.msg.activationId}"))
      else p.p.success(None)
      k += 1
    }
    val known = planned.flatMap(_._1)
    var r = 0
    while (r < nRel) {
      val f = out.get(5 * nPub + r)
      val e = known(r).entry
      keyUse.get(e.fullyQualifiedEntityName.asString).foreach(_.inFlight -= 1)
      if ((f & 1) != 0) // NS:103: concurrentSlotsMap(actionid) on a missing key
        logging.error(this, s"releaseInvoker: NoSuchElementException: key not found: ${e.fullyQualifiedEntityName}")
      if ((f & 2) != 0) // FS:48-50
        logging.error(this, s"releaseInvoker: Error: Maximum permit count exceeded (invoker ${known(r).invoker.toInt})")
      r += 1
    }
    batchNo += 1
    if (batchNo % 1024 == 0) dropColdKeys()
  }

  /** Keys idle for keyIdleBatches with no activation in flight: their handles go back to the engine
   *  (owgs_release_actions), which recycles handle and key ids; a later publish registers the action again. */
  private def dropColdKeys(): Unit = {
    val cold = keyUse.filter { case (_, u) => u.inFlight <= 0 && batchNo - u.lastBatch > keyIdleBatches }
    if (cold.isEmpty) return
    val hs = cold.values.flatMap(_.names.flatMap(handles.get)).toArray
    val rc = OwgsNative.releaseActions(ctx, hs, hs.length)
    if (rc < 0) logging.error(this, s"releaseActions: ${nativeError("owgs_release_actions", rc).getMessage}")
    else
      cold.foreach { case (key, u) =>
        u.names.foreach(handles.remove)
        byKey.remove(key)
        keyUse.remove(key)
      }
  }

  /** The single writer of the native context: drains the queue in batches (stream order is the sequential order).
   *  Any exception is contained to its batch, so the thread (and every later promise) survives. */
  private val batcher = new Thread(() => {
    val jobs = new java.util.ArrayList[Job](4096)
    while (true) {
      val first = queue.poll(1, TimeUnit.MILLISECONDS)
      if (first != null) {
        jobs.add(first)
        queue.drainTo(jobs, 4095)
        try runBatch(jobs)
        catch {
          case t: Throwable =>
            logging.error(this, s"owgs batcher: $t")
            val e = LoadBalancerException(s"scheduling batch failed: $t")
            jobs.forEach {
              case Pub(_, _, p) => p.tryFailure(e)
              case _               =>
            }
        }
        jobs.clear()
      }
    }
  }, "owgs-batcher")
  batcher.setDaemon(true)
  batcher.start()

  private def statusCode(s: InvokerState): Byte = s match {
    case InvokerState.Healthy      => 0
    case InvokerState.Unhealthy    => 1
    case InvokerState.Unresponsive => 2
    case InvokerState.Offline      => 3
  }

  /** Native handle of an action (registered on first use); a negative owgs error code is returned, not cached. */
  private def handleOf(ns: String, fqn: FullyQualifiedEntityName, memMb: Int, maxConc: Int, blackbox: Boolean): Int = {
    val key = fqn.asString
    val h = handles.get((ns, key)) match {
      case Some(h) => h
      case None =>
        val h = OwgsNative.registerAction(ctx, ns, fqn.copy(version = None).asString, key, memMb, maxConc, blackbox)
        if (h >= 0) {
          handles.update((ns, key), h)
          byKey.getOrElseUpdate(key, h)
          keyUse.getOrElseUpdate(key, new KeyUse(0, batchNo, mutable.ArrayBuffer.empty)).names += ((ns, key))
        }
        h
    }
    keyUse.get(key).foreach(_.lastBatch = batchNo)
    h
  }

  /** SCPB:169-205: capacity and health gauges of both pools, from the list the engine schedules against. */
  override protected def emitMetrics() = {
    super.emitMetrics()
    val p = pools
    def usableMb(s: IndexedSeq[InvokerHealth]) =
      s.foldLeft(0L)((total, curr) => if (curr.status.isUsable) curr.id.userMemory.toMB + total else total)
    MetricEmitter.emitGaugeMetric(INVOKER_TOTALMEM_BLACKBOX, usableMb(p.blackbox))
    MetricEmitter.emitGaugeMetric(INVOKER_TOTALMEM_MANAGED, usableMb(p.managed))
    MetricEmitter.emitGaugeMetric(HEALTHY_INVOKER_MANAGED, p.managed.count(_.status == Healthy))
    MetricEmitter.emitGaugeMetric(UNHEALTHY_INVOKER_MANAGED, p.managed.count(_.status == Unhealthy))
    MetricEmitter.emitGaugeMetric(UNRESPONSIVE_INVOKER_MANAGED, p.managed.count(_.status == Unresponsive))
    MetricEmitter.emitGaugeMetric(OFFLINE_INVOKER_MANAGED, p.managed.count(_.status == Offline))
    MetricEmitter.emitGaugeMetric(HEALTHY_INVOKER_BLACKBOX, p.blackbox.count(_.status == Healthy))
    MetricEmitter.emitGaugeMetric(UNHEALTHY_INVOKER_BLACKBOX, p.blackbox.count(_.status == Unhealthy))
    MetricEmitter.emitGaugeMetric(UNRESPONSIVE_INVOKER_BLACKBOX, p.blackbox.count(_.status == Unresponsive))
    MetricEmitter.emitGaugeMetric(OFFLINE_INVOKER_BLACKBOX, p.blackbox.count(_.status == Offline))
  }

  // state updates go through the batching thread too, so they are serialized with publishes exactly like the
  // reference's monitor actor serializes updateInvokers / updateCluster (SCPB:210-250)
  private val monitor = actorSystem.actorOf(Props(new Actor {
    override def preStart(): Unit = {
      cluster.foreach(_.subscribe(self, classOf[MemberEvent], classOf[ReachabilityEvent]))
    }

    // all members of the cluster that are available
    var availableMembers = Set.empty[Member]

    override def receive: Receive = {
      case CurrentInvokerPoolState(newState) =>
        queue.put(Inv(newState))
      case CurrentClusterState(members, _, _, _, _) =>
        availableMembers = members.filter(_.status == MemberStatus.Up)
        queue.put(Clu(availableMembers.size))
      case event: ClusterDomainEvent =>
        availableMembers = event match {
          case MemberUp(member)          => availableMembers + member
          case ReachableMember(member)   => availableMembers + member
          case MemberRemoved(member, _)  => availableMembers - member
          case UnreachableMember(member) => availableMembers - member
          case _                         => availableMembers
        }
        queue.put(Clu(availableMembers.size))
    }
  }))

  override def invokerHealth(): Future[IndexedSeq[InvokerHealth]] = Future.successful(pools.all)
  override def clusterSize: Int = _clusterSize

  /** SCPB:257-317 with the schedule() half (SCPB:260-290) executed natively in batches. */
  override def publish(action: ExecutableWhiskActionMetaData, msg: ActivationMessage)(
    implicit transid: TransactionId): Future[Future[Either[ActivationId, WhiskActivation]]] = {
    val isBlackboxInvocation = action.exec.pull
    val actionType = if (!isBlackboxInvocation) "managed" else "blackbox"
    val p = Promise[Option[(InvokerInstanceId, Boolean)]]()
    queue.put(Pub(action, msg, p))
    p.future.flatMap {
      case Some((invoker, overload)) =>
        if (overload)
          MetricEmitter.emitCounterMetric(
            if (isBlackboxInvocation) LoggingMarkers.BLACKBOX_SYSTEM_OVERLOAD else LoggingMarkers.MANAGED_SYSTEM_OVERLOAD)
        // SCPB:293-301
        val memoryLimit = action.limits.memory
        val memoryLimitInfo = if (memoryLimit == MemoryLimit()) { "std" } else { "non-std" }
        val timeLimit = action.limits.timeout
        val timeLimitInfo = if (timeLimit == TimeLimit()) { "std" } else { "non-std" }
        logging.info(
          this,
          s"scheduled activation ${msg.activationId}, action '${msg.action.asString}' ($actionType), ns '${msg.user.namespace.name.asString}', mem limit ${memoryLimit.megabytes} MB (${memoryLimitInfo}), time limit ${timeLimit.duration.toMillis} ms (${timeLimitInfo}) to ${invoker}")
        val activationResult = setupActivation(msg, action, invoker)
        sendActivationToInvoker(messageProducer, msg, invoker).map(_ => activationResult)
      case None =>
        // SCPB:305-316: report the state of all invokers of the pool
        val p = pools
        val invokersToUse = if (!isBlackboxInvocation) p.managed else p.blackbox
        val invokerStates = invokersToUse.foldLeft(Map.empty[InvokerState, Int]) { (agg, curr) =>
          agg + (curr.status -> (agg.getOrElse(curr.status, 0) + 1))
        }
        logging.error(
          this,
          s"failed to schedule activation ${msg.activationId}, action '${msg.action.asString}' ($actionType), ns '${msg.user.namespace.name.asString}' - invokers to use: $invokerStates")
        Future.failed(LoadBalancerException("No invokers available"))
    }
  }

  override val invokerPool: ActorRef = invokerPoolFactory.createInvokerPool(
    actorSystem, messagingProvider, messageProducer, sendActivationToInvoker, Some(monitor))

  /** SCPB:327-331: releaseConcurrent through the native context. */
  override protected def releaseInvoker(invoker: InvokerInstanceId, entry: ActivationEntry): Unit =
    queue.put(Rel(invoker, entry))
}

object GpuShardingContainerPoolBalancer extends LoadBalancerProvider {
  override def instance(whiskConfig: WhiskConfig, instance: ControllerInstanceId)(
    implicit actorSystem: ActorSystem, logging: Logging, materializer: ActorMaterializer): LoadBalancer = {
    // the same invoker-supervision wiring the reference provider builds (SCPB:341-358): health pings from the
    // "health" topic drive InvokerPool, which reports CurrentInvokerPoolState to our monitor actor
    val pools = new InvokerPoolFactory {
      override def createInvokerPool(f: ActorRefFactory, mp: MessagingProvider, producer: MessageProducer,
                                     send: (MessageProducer, ActivationMessage, InvokerInstanceId) => Future[RecordMetadata],
                                     monitor: Option[ActorRef]): ActorRef = {
        InvokerPool.prepare(instance, WhiskEntityStore.datastore())
        val healthFeed = mp.getConsumer(whiskConfig, s"health${instance.asString}", "health", maxPeek = 128)
        f.actorOf(InvokerPool.props((af, i) => af.actorOf(InvokerActor.props(i, instance)),
          (m, i) => send(producer, m, i), healthFeed, monitor))
      }
    }
    new GpuShardingContainerPoolBalancer(whiskConfig, instance, createFeedFactory(whiskConfig, instance), pools)
  }

  def requiredProperties: Map[String, String] = kafkaHosts
}

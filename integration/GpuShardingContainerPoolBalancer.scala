/*
 * Drop-in LoadBalancerProvider for the MI355X engine (SOURCE ONLY: this image has no JDK/scalac, see DESIGN.md).
 *
 * A maintainer adds this file to core/controller/src/main/scala/org/apache/openwhisk/core/loadBalancer/ and selects
 * it with   whisk.spi.LoadBalancerProvider = org.apache.openwhisk.core.loadBalancer.GpuShardingContainerPoolBalancer
 * (common/scala/src/main/resources/reference.conf:26, or CONFIG_whisk_spi_LoadBalancerProvider).
 *
 * Everything except the scheduling state stays as in ShardingContainerPoolBalancer (SCPB): CommonLoadBalancer keeps
 * activation bookkeeping, the Kafka send, the ack feed and processCompletion; the monitor actor keeps forwarding
 * CurrentInvokerPoolState and cluster membership.  publish() enqueues into a single batching thread that owns the
 * native context (single writer, owgs.h "Threading"), which calls owgs_publish_batch and completes the promises in
 * stream order; releaseInvoker() enqueues into the same thread (owgs_release_batch).
 */
package org.apache.openwhisk.core.loadBalancer

import java.util.concurrent.{ArrayBlockingQueue, TimeUnit}

import akka.actor.{Actor, ActorRef, ActorRefFactory, ActorSystem, Props}
import akka.stream.ActorMaterializer
import org.apache.kafka.clients.producer.RecordMetadata
import org.apache.openwhisk.common._
import org.apache.openwhisk.core.WhiskConfig
import org.apache.openwhisk.core.WhiskConfig._
import org.apache.openwhisk.core.connector._
import org.apache.openwhisk.core.entity._
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
  @native def publishBatch(ctx: Long, actions: Array[Int], seq: Array[Long], n: Int, outInvoker: Array[Int],
                           outFlags: Array[Byte]): Int
  @native def releaseBatch(ctx: Long, invokers: Array[Int], actions: Array[Int], n: Int, outFlags: Array[Byte]): Int
  @native def lastError(ctx: Long): String
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

  // device and overload-RNG seed of this controller: whisk.loadbalancer.gpu.{device, rng-seed} (optional keys)
  private val gpuConfig = actorSystem.settings.config
  private def cfgInt(k: String, d: Int): Int = if (gpuConfig.hasPath(k)) gpuConfig.getInt(k) else d
  private def cfgLong(k: String, d: Long): Long = if (gpuConfig.hasPath(k)) gpuConfig.getLong(k) else d
  private val ctx = OwgsNative.create(lbConfig.managedFraction, lbConfig.blackboxFraction,
    MemoryLimit.MIN_MEMORY.toBytes, 1, cfgInt("whisk.loadbalancer.gpu.device", 0),
    cfgLong("whisk.loadbalancer.gpu.rng-seed", controllerInstance.asString.hashCode.toLong))
  require(ctx != 0L, "owgs_create failed (no MI355X visible or libowgs.so missing)")

  // (invoking namespace, fqn@version) -> native action handle (registered once); fqn@version -> a handle of that
  // action for releases (a release only needs the NestedSemaphore key and the limits, NS:98-113)
  private val handles = mutable.HashMap.empty[(String, String), Int]
  private val byKey = mutable.HashMap.empty[String, Int]
  @volatile private var invokerList: IndexedSeq[InvokerHealth] = IndexedSeq.empty
  // userMemory by invoker id (ids are dense: InvokerPool pads the list by id, InvokerSupervision.scala:191-207)
  @volatile private var invokerMemoryById: Array[ByteSize] = Array.empty
  @volatile private var _clusterSize = 1

  private sealed trait Job
  private case class Pub(action: ExecutableWhiskActionMetaData, msg: ActivationMessage, seq: Long,
                         p: Promise[Option[(InvokerInstanceId, Boolean)]]) extends Job
  private case class Rel(invoker: InvokerInstanceId, entry: ActivationEntry) extends Job
  private case class Inv(state: IndexedSeq[InvokerHealth]) extends Job
  private case class Clu(size: Int) extends Job

  private val queue = new ArrayBlockingQueue[Job](1 << 16)
  private var seqNo = 0L

  private def nativeError(what: String, rc: Int): LoadBalancerException =
    LoadBalancerException(s"$what failed ($rc): ${OwgsNative.lastError(ctx)}")

  /** One drained batch of jobs, in queue order (the sequential order the engine replays). */
  private def runBatch(jobs: java.util.ArrayList[Job]): Unit = {
    var i = 0
    while (i < jobs.size) {
      jobs.get(i) match {
        case Inv(s) =>
          val rc = OwgsNative.updateInvokers(ctx, s.map(_.id.toInt).toArray, s.map(_.id.userMemory.toBytes).toArray,
            s.map(h => statusCode(h.status)).toArray)
          if (rc < 0) logging.error(this, s"updateInvokers: ${nativeError("owgs_update_invokers", rc).getMessage}")
          i += 1
        case Clu(n) =>
          val rc = OwgsNative.updateCluster(ctx, n)
          if (rc < 0) logging.error(this, s"updateCluster: ${nativeError("owgs_update_cluster", rc).getMessage}")
          i += 1
        case _ =>
          // maximal run of releases followed by publishes: one native call each, order preserved
          val rels = mutable.ArrayBuffer.empty[Rel]
          while (i < jobs.size && jobs.get(i).isInstanceOf[Rel]) { rels += jobs.get(i).asInstanceOf[Rel]; i += 1 }
          if (rels.nonEmpty) releaseRun(rels)
          val pubs = mutable.ArrayBuffer.empty[Pub]
          while (i < jobs.size && jobs.get(i).isInstanceOf[Pub]) { pubs += jobs.get(i).asInstanceOf[Pub]; i += 1 }
          if (pubs.nonEmpty) publishRun(pubs)
      }
    }
  }

  /** releaseInvoker (SCPB:327-331) for a run of completions.  What the reference would throw from
   *  NestedSemaphore.releaseConcurrent / ForcibleSemaphore.release is logged per release (processCompletion's
   *  future fails there too); a native error fails nothing else. */
  private def releaseRun(rels: mutable.ArrayBuffer[Rel]): Unit = {
    val known = rels.filter(r => byKey.contains(r.entry.fullyQualifiedEntityName.asString))
    val inv = known.map(_.invoker.toInt).toArray
    val act = known.map(r => byKey(r.entry.fullyQualifiedEntityName.asString)).toArray
    val flags = new Array[Byte](inv.length)
    val rc = OwgsNative.releaseBatch(ctx, inv, act, inv.length, flags)
    if (rc < 0) {
      logging.error(this, s"releaseInvoker: ${nativeError("owgs_release_batch", rc).getMessage}")
    } else {
      var k = 0
      while (k < flags.length) {
        val f = flags(k)
        val e = known(k).entry
        if ((f & 1) != 0) // NS:103: concurrentSlotsMap(actionid) on a missing key
          logging.error(this, s"releaseInvoker: NoSuchElementException: key not found: ${e.fullyQualifiedEntityName}")
        if ((f & 2) != 0) // FS:48-50
          logging.error(this, s"releaseInvoker: Error: Maximum permit count exceeded (invoker ${inv(k)})")
        k += 1
      }
    }
  }

  /** The schedule() half of publish (SCPB:260-290) for a run of activations; on a native error every promise of the
   *  run fails with LoadBalancerException (nothing was acquired: the native call is all-or-nothing). */
  private def publishRun(pubs: mutable.ArrayBuffer[Pub]): Unit = {
    val act = new Array[Int](pubs.length)
    var bad = false
    var k = 0
    while (k < pubs.length) {
      val p = pubs(k)
      val h = handleOf(p.msg.user.namespace.name.asString, p.action.fullyQualifiedName(true),
        p.action.limits.memory.megabytes, p.action.limits.concurrency.maxConcurrent, p.action.exec.pull)
      if (h < 0) bad = true
      act(k) = h
      k += 1
    }
    if (bad) {
      // registration failed for some action: fail those promises, schedule the rest in order
      val (failed, ok) = pubs.zip(act).partition(_._2 < 0)
      failed.foreach { case (p, h) => p.p.failure(nativeError("owgs_register_actions", h)) }
      if (ok.nonEmpty) publishRun(ok.map(_._1))
      return
    }
    val out = new Array[Int](act.length)
    val flags = new Array[Byte](act.length)
    val rc = OwgsNative.publishBatch(ctx, act, pubs.map(_.seq).toArray, act.length, out, flags)
    if (rc < 0) {
      val e = nativeError("owgs_publish_batch", rc)
      pubs.foreach(_.p.failure(e))
      return
    }
    val mem = invokerMemoryById
    pubs.zipWithIndex.foreach { case (p, k) =>
      val id = out(k)
      val r =
        if (id >= 0) Some((InvokerInstanceId(id, userMemory = if (id < mem.length) mem(id) else 0.B), (flags(k) & 1) != 0))
        else None // -1: no invokers; -2: the reference's schedule() would have thrown
      p.p.success(r)
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
              case Pub(_, _, _, p) => p.tryFailure(e)
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
  private def handleOf(ns: String, fqn: FullyQualifiedEntityName, memMb: Int, maxConc: Int, blackbox: Boolean): Int =
    handles.get((ns, fqn.asString)) match {
      case Some(h) => h
      case None =>
        val h = OwgsNative.registerAction(ctx, ns, fqn.copy(version = None).asString, fqn.asString, memMb, maxConc,
          blackbox)
        if (h >= 0) {
          handles.update((ns, fqn.asString), h)
          byKey.getOrElseUpdate(fqn.asString, h)
        }
        h
    }

  // state updates go through the batching thread too, so they are serialized with publishes exactly like the
  // reference's monitor actor serializes updateInvokers / updateCluster (SCPB:210-250)
  private val monitor = actorSystem.actorOf(Props(new Actor {
    private var members = Set.empty[akka.cluster.Member]
    override def preStart(): Unit =
      if (actorSystem.settings.config.getStringList("akka.cluster.seed-nodes").size > 0)
        akka.cluster.Cluster(actorSystem)
          .subscribe(self, classOf[akka.cluster.ClusterEvent.MemberEvent], classOf[akka.cluster.ClusterEvent.ReachabilityEvent])
    override def receive: Receive = {
      case CurrentInvokerPoolState(newState) =>
        invokerList = newState
        val mem = new Array[ByteSize](if (newState.isEmpty) 0 else newState.map(_.id.toInt).max + 1)
        java.util.Arrays.fill(mem.asInstanceOf[Array[AnyRef]], 0.B)
        newState.foreach(h => mem(h.id.toInt) = h.id.userMemory)
        invokerMemoryById = mem
        queue.put(Inv(newState))
      case akka.cluster.ClusterEvent.CurrentClusterState(ms, _, _, _, _) =>
        members = ms.filter(_.status == akka.cluster.MemberStatus.Up)
        _clusterSize = math.max(1, members.size); queue.put(Clu(members.size))
      case e: akka.cluster.ClusterEvent.ClusterDomainEvent =>
        members = e match {
          case akka.cluster.ClusterEvent.MemberUp(m)          => members + m
          case akka.cluster.ClusterEvent.ReachableMember(m)   => members + m
          case akka.cluster.ClusterEvent.MemberRemoved(m, _)  => members - m
          case akka.cluster.ClusterEvent.UnreachableMember(m) => members - m
          case _                                             => members
        }
        _clusterSize = math.max(1, members.size); queue.put(Clu(members.size))
    }
  }))

  override def invokerHealth(): Future[IndexedSeq[InvokerHealth]] = Future.successful(invokerList)
  override def clusterSize: Int = _clusterSize

  /** SCPB:257-317 with the schedule() half (SCPB:260-290) executed natively in batches. */
  override def publish(action: ExecutableWhiskActionMetaData, msg: ActivationMessage)(
    implicit transid: TransactionId): Future[Future[Either[ActivationId, WhiskActivation]]] = {
    val p = Promise[Option[(InvokerInstanceId, Boolean)]]()
    val s = synchronized { seqNo += 1; seqNo }
    queue.put(Pub(action, msg, s, p))
    p.future.flatMap {
      case Some((invoker, overload)) =>
        if (overload)
          MetricEmitter.emitCounterMetric(
            if (action.exec.pull) LoggingMarkers.BLACKBOX_SYSTEM_OVERLOAD else LoggingMarkers.MANAGED_SYSTEM_OVERLOAD)
        val activationResult = setupActivation(msg, action, invoker)
        sendActivationToInvoker(messageProducer, msg, invoker).map(_ => activationResult)
      case None => Future.failed(LoadBalancerException("No invokers available"))
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

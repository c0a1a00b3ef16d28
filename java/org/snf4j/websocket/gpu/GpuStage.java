/*
 * A decoder after "ws-decoder" that the MI355X batch can run itself: the stages
 * wsg_batcher_set_stages chains behind the device decode (inflate, the UTF-8
 * validator, the aggregator).  When the session's first bytes arrive,
 * GpuFrameDecoder takes the GPU stages that directly follow it, in the pipeline
 * order the reference builds, into its batch and marks them batched: from then on
 * its deliver() skips them.  A stage that is not batched (added later, or behind
 * another decoder) runs its reference decoder on each frame instead.
 */
package org.snf4j.websocket.gpu;

interface GpuStage {

	/** The stage runs inside the decoder's device batch from now on. */
	void setBatched();

	boolean isBatched();
}

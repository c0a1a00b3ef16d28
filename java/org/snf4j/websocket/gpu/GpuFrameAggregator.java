/*
 * FrameAggregator (FrameAggregator.java:40-104) on the MI355X: in the decoder's
 * device batch (wsg_aggregate_batch_*, aggregate.hip) when it directly follows the
 * GPU decode stages; the reference FrameAggregator otherwise.  The batch delivers
 * a fragmented message as one AggregatedTextFrame / AggregatedBinaryFrame, its
 * bytes from earlier batches kept by the native batcher as PayloadAggregator keeps
 * its fragment list (PayloadAggregator.java:34).
 */
package org.snf4j.websocket.gpu;

import java.util.List;

import org.snf4j.core.codec.IDecoder;
import org.snf4j.core.session.ISession;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.FrameAggregator;

public class GpuFrameAggregator implements IDecoder<Frame, Frame>, GpuStage {

	/** The pipeline key GpuWebSocketSessionConfig installs it under. */
	public static final String KEY = "ws-aggregator";

	final int maxAggregatedLength;
	private final FrameAggregator fallback;
	private boolean batched;

	public GpuFrameAggregator(int maxAggregatedLength) {
		this.maxAggregatedLength = maxAggregatedLength;
		this.fallback = new FrameAggregator(maxAggregatedLength);
	}

	@Override
	public Class<Frame> getInboundType() {
		return Frame.class;
	}

	@Override
	public Class<Frame> getOutboundType() {
		return Frame.class;
	}

	@Override
	public void setBatched() {
		batched = true;
	}

	@Override
	public boolean isBatched() {
		return batched;
	}

	@Override
	public void decode(ISession session, Frame frame, List<Frame> out) throws Exception {
		if (batched)
			out.add(frame);  // (aggregated in the device batch)
		else
			fallback.decode(session, frame, out);
	}
}

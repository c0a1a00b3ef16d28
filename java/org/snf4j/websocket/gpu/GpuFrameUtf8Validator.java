/*
 * The "ws-utf8-validator" stage (FrameUtf8Validator.java:40-100) on the MI355X.
 *
 * Directly behind the GPU decoder it is the UTF-8 check fused into the decode
 * kernels (k_piecesN); behind the GPU inflate stage it is the validator stage of
 * the same device batch (wsg_validate_batch_*, k_vparse/k_vlink): either way
 * GpuFrameDecoder runs it and this object only marks the place.  Not batched, it
 * is the reference FrameUtf8Validator.
 */
package org.snf4j.websocket.gpu;

import java.util.List;

import org.snf4j.core.codec.IDecoder;
import org.snf4j.core.session.ISession;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.FrameUtf8Validator;

public class GpuFrameUtf8Validator implements IDecoder<Frame, Frame>, GpuStage {

	private final FrameUtf8Validator fallback = new FrameUtf8Validator();
	private boolean batched;

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
			out.add(frame);  // (validated in the device batch)
		else
			fallback.decode(session, frame, out);
	}
}
